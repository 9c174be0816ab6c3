// spmm_bench.cpp -- benchmark harness driving one Matrix_Format plugin (here the HIP plugin).
//
// Keeps the reference harness contract (benchmark_code/CPU/AMD/spmv_code_bench/spmv_bench.cpp:564-1035) so the
// existing run scripts drive it unchanged:
//   env   NUM_COLS (= K), USE_ARTIFICIAL_MATRICES (0 = argv[1] is a .mtx path, 1 = argv holds the 11 generator
//         parameters), USE_DLCM_MATRICES (1 = argv[1] is a DLMC .smtx path; values seeded U[-1,1)),
//         USE_PROCESSES (fork replicas: not supported, must be 0), COOLDOWN
//   argv  none -> print the CSV labels and exit (:606-610); a path; or 11 generator fields [+ name] (:851-868)
//   out   log lines on stdout, ONE CSV row on stderr (:478 / :555), the accuracy report on stdout (:187-203)
//   flow  x = B = 1.0 (:901), y = 0 (:907), csr_to_format (:996), 100 warm-up spmm calls (:316-320), timed calls
//         (:365-378), gflops = 2*nnz*K/t (:115-117), CheckAccuracy for file matrices (:480)
// Deliberate fixes of reference quirks: missing env variables get defaults instead of
// atoi(NULL) (9); B/C sizes use 64-bit products (3); a single quoted generator line is word-split (10); the
// reported time is the MEDIAN of SPMM_TIMED_LOOPS calls (default 1, the reference's min_num_loops) rather than
// the last call times the loop count (4).  Added env: SPMM_WARMUP (default 100), SPMM_TIMED_LOOPS (default 1),
// SPMM_B_RANDOM=1 (B = drand48 stream seeded 42 instead of 1.0), SPMM_CHECK=1 (accuracy report for synthetic
// matrices too).  Energy (RAPL) is out of scope: W_avg and J_estimated print 0.
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/spmm_host.h"
#include "matrix_format.h"

namespace {

long env_long(const char *name, long dflt) {
    const char *v = getenv(name);
    return (v && *v) ? atol(v) : dflt;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double gflops(double t, long nnz, long k, long loops) { return t > 0 ? (double)nnz * 2e-9 * (double)k / t * loops : 0; }

void print_labels(bool artificial) {
    std::string s;
    if (!artificial) {
        s = "matrix_name,num_threads,input_columns,csr_m,csr_k,csr_nnz,time,gflops,csr_mem_footprint,m,n,nnz";
    } else {
        s = "matrix_name,distribution,placement,seed,nr_rows,nr_cols,nr_nzeros,density,mem_footprint,mem_range,"
            "avg_nnz_per_row,std_nnz_per_row,avg_bw,std_bw,avg_bw_scaled,std_bw_scaled,avg_sc,std_sc,avg_sc_scaled,"
            "std_sc_scaled,skew,avg_num_neighbours,cross_row_similarity,format_name,time,gflops,W_avg,J_estimated";
    }
    char buf[4096];
    int w = statistics_print_labels(buf, sizeof(buf));
    if (w > 0) s += std::string(buf, (size_t)w);
    fprintf(stderr, "%s\n", s.c_str());
}

}  // namespace

int main(int argc, char **argv) {
    const long K = env_long("NUM_COLS", 32);
    const bool artificial = env_long("USE_ARTIFICIAL_MATRICES", 0) != 0;
    const long warmup = env_long("SPMM_WARMUP", 100);
    const long loops = std::max(1L, env_long("SPMM_TIMED_LOOPS", 1));
    if (env_long("USE_PROCESSES", 0) != 0) {
        fprintf(stderr, "USE_PROCESSES=1 (fork replicas) is not supported by the HIP harness\n");
        return EXIT_FAILURE;
    }
    int nthreads = 1;
#pragma omp parallel
    nthreads = omp_get_max_threads();
    printf("max threads %d\n", nthreads);
    if (argc == 1) {
        print_labels(artificial);
        return 0;
    }
    if (K < 1) {
        fprintf(stderr, "NUM_COLS must be >= 1\n");
        return EXIT_FAILURE;
    }

    spmm_csr_t A{};
    spmm_features_t F{};
    spmm_gen_params_t P{};
    std::string matrix_name;
    double t0 = now_s();
    if (!artificial) {
        matrix_name = argv[1];
        char field[32] = {0};
        int sym = 0;
        // USE_DLCM_MATRICES=1: argv[1] is a DLMC .smtx file, used as stored (spmv_bench.cpp:667-696,769-801)
        int st = env_long("USE_DLCM_MATRICES", 0) != 0 ? spmm_host_smtx_read(argv[1], 42, &A)
                                                        : spmm_host_mtx_read(argv[1], &A, field, sizeof(field), &sym);
        if (st) {
            fprintf(stderr, "error reading '%s' (status %d)\n", argv[1], st);
            return EXIT_FAILURE;
        }
        printf("time read + coo to csr: %lf\n", now_s() - t0);
    } else {
        std::string line;
        int consumed = 0;
        if (argc >= 12) {
            for (int i = 1; i <= 11; ++i) line += std::string(argv[i]) + " ";
            consumed = 11;
        } else {
            line = argv[1];  // a whole generator line passed as one argv (CPU/AMD run.sh:678)
            consumed = 1;
        }
        if (spmm_host_parse_gen_line(line.c_str(), &P) != SPMM_HOST_OK) {
            fprintf(stderr, "cannot parse generator parameters: '%s'\n", line.c_str());
            return EXIT_FAILURE;
        }
        int st = spmm_host_generate(&P, &A);
        if (st) {
            fprintf(stderr, "generator failed (status %d)\n", st);
            return EXIT_FAILURE;
        }
        spmm_host_features(&A, &F);
        if (argc > consumed + 1)
            matrix_name = std::string(argv[consumed + 1]) + "_artificial";
        else
            matrix_name = std::to_string(A.m) + "_" + std::to_string(A.ncols) + "_" + std::to_string(A.nnz);
        printf("time generate artificial matrix: %lf\n", now_s() - t0);
    }

    const long m = A.m, ncols = A.ncols, nnz = A.nnz;
    // harness-owned arrays, 64-B aligned like aligned_alloc(64, ...) at spmv_bench.cpp:871-883
    auto alloc64 = [](size_t bytes) { return aligned_alloc(64, ((std::max<size_t>(bytes, 64) + 63) / 64) * 64); };
    INT_T *csr_ia = (INT_T *)alloc64((size_t)(m + 1) * sizeof(INT_T));
    INT_T *csr_ja = (INT_T *)alloc64((size_t)nnz * sizeof(INT_T));
    ValueType *csr_a = (ValueType *)alloc64((size_t)nnz * sizeof(ValueType));
    memcpy(csr_ia, A.row_ptr, (size_t)(m + 1) * sizeof(INT_T));
    memcpy(csr_ja, A.col_idx, (size_t)nnz * sizeof(INT_T));
    for (long i = 0; i < nnz; ++i) csr_a[i] = (ValueType)A.values[i];

    const size_t xn = (size_t)ncols * (size_t)K, yn = (size_t)m * (size_t)K;
    std::vector<double> x_ref(xn, 1.0);
    if (env_long("SPMM_B_RANDOM", 0)) spmm_host_drand48_fill(42, x_ref.data(), (int64_t)xn);
    ValueType *x = (ValueType *)alloc64(xn * sizeof(ValueType));
    ValueType *y = (ValueType *)alloc64(yn * sizeof(ValueType));
    for (size_t i = 0; i < xn; ++i) x[i] = (ValueType)x_ref[i];
    memset(y, 0, yn * sizeof(ValueType));

    t0 = now_s();
    struct Matrix_Format *MF = csr_to_format(csr_ia, csr_ja, csr_a, m, ncols, nnz, (int)K);
    printf("time convert to format: %lf\n", now_s() - t0);

    t0 = now_s();
    for (long it = 0; it < warmup; ++it) MF->spmm(x, y, (INT_T)K);
    double tw = now_s() - t0;
    printf("time warm up:%lf s (%lf GFLOPS/s)\n", tw, gflops(tw, nnz, K, warmup));

    MF->statistics_start();
    std::vector<double> times;
    for (long it = 0; it < loops; ++it) {
        t0 = now_s();
        MF->spmm(x, y, (INT_T)K);
        times.push_back(now_s() - t0);
    }
    std::vector<double> sorted = times;
    std::sort(sorted.begin(), sorted.end());
    const double time = sorted[sorted.size() / 2];
    const double gf = gflops(time, nnz, K, 1);
    printf("number of loops = %ld\n", loops);
    printf("threads %d time spmm:%lf s (%lf GFLOPS/s) min %lf s\n", nthreads, time, gf, sorted.front());

    char stats[4096];
    int sw = MF->statistics_print_data(stats, sizeof(stats));
    std::string st_s = sw > 0 ? std::string(stats, (size_t)sw) : std::string();
    char row[8192];
    if (!artificial) {
        snprintf(row, sizeof(row), "%s,%d,%ld,%ld,%ld,%ld,%lf,%lf,%lf,%d,%d,%d%s", matrix_name.c_str(), nthreads, K, m,
                 ncols, nnz, time, gf, MF->csr_mem_footprint / (1024 * 1024), MF->m, MF->n, MF->nnz, st_s.c_str());
    } else {
        snprintf(row, sizeof(row),
                 "synthetic,%s,%s,%lld,%lld,%lld,%lld,%lf,%lf,%s,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%lf,%s,%lf,"
                 "%lf,%lf,%lf%s",
                 P.distribution, P.placement, (long long)P.seed, (long long)F.nr_rows, (long long)F.nr_cols,
                 (long long)F.nr_nzeros, F.density, F.mem_footprint, F.mem_range, F.avg_nnz_per_row, F.std_nnz_per_row,
                 F.avg_bw, F.std_bw, F.avg_bw_scaled, F.std_bw_scaled, F.avg_sc, F.std_sc, F.avg_sc_scaled,
                 F.std_sc_scaled, F.skew, F.avg_num_neighbours, F.cross_row_similarity, MF->format_name, time, gf, 0.0,
                 0.0, st_s.c_str());
    }
    fprintf(stderr, "%s\n", row);

    if (!artificial || env_long("SPMM_CHECK", 0)) {
        const double eps = (sizeof(ValueType) == 8) ? 1e-10 : 1e-7;  // spmv_bench.cpp:125-129
        double out[11];
        spmm_host_check_accuracy(A.row_ptr, A.col_idx, A.values, m, ncols, x_ref.data(), (int32_t)K, y,
                                 sizeof(ValueType) == 8 ? 0 : 1, eps, out);
        if (out[0] > eps) printf("Test failed! (%g)\n", out[0]);
        printf("errors spmv: mae=%g, max_ae=%g, mse=%g, mape=%g, smape=%g, lnQ_error=%g, mlare=%g, gmare=%g\n", out[1],
               out[2], out[3], out[4], out[5], out[6], out[7], out[8]);
        printf("normwise check (eps=%g): failing entries=%.0f, worst |y-gold|/max(|gold|,sum|ab|)=%g\n", eps, out[9],
               out[10]);
    }
    if (env_long("COOLDOWN", 0) == 1) {
        printf("cooldown\n");
    }
    delete MF;  // virtual destructor: the plugin frees csr_ia/csr_ja/csr_a and its device state
    free(x);
    free(y);
    spmm_host_csr_free(&A);
    return 0;
}

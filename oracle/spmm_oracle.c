/*
 * oracle/spmm_oracle.c -- CPU restatement of the reference's CSR SpMM hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (spmm-research_amd/, include/) links, loads or
 * calls this file.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and
 * only as the checker / the timed CPU baseline.
 *
 * Parity pinning: every function here is checked in tests/test_oracle_golden.py against golden vectors
 * produced by the reference itself (its own sources compiled by oracle/Makefile into oracle/_ref/, driven
 * by oracle/ref_driver.cpp; fixtures + generating script in tests/golden/).
 *
 * Restated functions (reference paths relative to /root/reference):
 *   oracle_spmm_csr_{d,f}     benchmark_code/CPU/AMD/spmv_code_bench/spmm_kernel_csr.cpp:70-96 (compute_csr)
 *   oracle_binary_search      lib/macros/macrolib.h:471-524 (__binary_search, default cmp/dist :440-448)
 *   oracle_partition          lib/parallel_util.h:141-165 (loop_partitioner_balance_prefix_sums)
 *   oracle_gold_{d,f}         benchmark_code/CPU/AMD/spmv_code_bench/spmv_bench.cpp:121-160 (CheckAccuracy gold:
 *                             __float128 Kahan-compensated row sums)
 *   oracle_check_accuracy     spmv_bench.cpp:162-203 (max relative diff over y_gold > eps; 8 metrics from
 *                             lib/array_metrics.c:1472 mae, :1528 max_ae, :1586 mse, :1643/1696 mape,
 *                             :1754/1810 smape, :1925 lnQ, :1996 mlare, :2112 gmare)
 *   oracle_coo_to_csr         lib/storage_formats/csr/csr_gen.c:163-217 (bucket by row, scatter, sort columns)
 *   oracle_sddmm_{d,f}        benchmark_code/CPU/AMD/pipeline_code_bench/sddmm_taco_naive.cpp:98-140 (compute2) and
 *                             :280-290 (compute_csr zeroes y first): the sparse-attention pipeline's SDDMM
 *   oracle_softmax_{d,f}      pipeline_code_bench/sddmm_taco_naive.cpp:191-209 (softmax over all nonzeros)
 *   The pipeline restatements are pinned by the reference's own gold (sddmm_bench.cpp:250-280 computes the same
 *   row-i-of-K product) and by tests/test_pipeline.py; the reference pipeline plugin itself needs Intel MKL
 *   (absent here), so no reference build pins them bit for bit.
 *
 * Summation order: compute_csr accumulates each output entry left-to-right over the row's nonzeros, starting
 * from 0.  Compiled with the reference flags on an FMA-capable x86 (-O3 -march=...), GCC contracts
 * `val = a*x; sum += val` into one fused multiply-add per nonzero; this restatement writes that fma()
 * explicitly so its bits do not depend on the compiler.  test_oracle_golden checks it bit-for-bit against the
 * compiled reference.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <quadmath.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------------------------------------------------
 * compute_csr  (spmm_kernel_csr.cpp:70-96)
 *   B = x: column-major, column n at x[n*ncols .. n*ncols+ncols)   (:88)
 *   C = y: row-major, y[i*k + n]                                   (:93)
 * Loop order kept: outer over the k columns, OpenMP static over rows inside (one implicit barrier per column).
 * ------------------------------------------------------------------------------------------------------- */
void oracle_spmm_csr_d(const int32_t *ia, const int32_t *ja, const double *a, int64_t m, int64_t ncols,
                       const double *x, double *y, int32_t k, int32_t nthreads)
{
#ifdef _OPENMP
	if (nthreads <= 0) nthreads = omp_get_max_threads();
	#pragma omp parallel num_threads(nthreads)
#endif
	{
		for (int64_t n = 0; n < k; n++) {
#ifdef _OPENMP
			#pragma omp for schedule(static)
#endif
			for (int64_t i = 0; i < m; i++) {
				double sum = 0;
				for (int64_t j = ia[i]; j < ia[i + 1]; j++)
					sum = fma(a[j], x[n * ncols + ja[j]], sum);
				y[i * k + n] = sum;
			}
		}
	}
}

void oracle_spmm_csr_f(const int32_t *ia, const int32_t *ja, const float *a, int64_t m, int64_t ncols,
                       const float *x, float *y, int32_t k, int32_t nthreads)
{
#ifdef _OPENMP
	if (nthreads <= 0) nthreads = omp_get_max_threads();
	#pragma omp parallel num_threads(nthreads)
#endif
	{
		for (int64_t n = 0; n < k; n++) {
#ifdef _OPENMP
			#pragma omp for schedule(static)
#endif
			for (int64_t i = 0; i < m; i++) {
				float sum = 0;
				for (int64_t j = ia[i]; j < ia[i + 1]; j++)
					sum = fmaf(a[j], x[n * ncols + ja[j]], sum);
				y[i * k + n] = sum;
			}
		}
	}
}

/* ---------------------------------------------------------------------------------------------------------
 * binary_search  (macrolib.h:471-524 with the default comparator/distance, :440-448)
 * Returns the index in A[lo..hi] equal to target, else the nearer of the two bracketing indices (ties -> the
 * upper one); clamps to lo/hi when target is outside the range.
 * ------------------------------------------------------------------------------------------------------- */
static int cmp_i64(int64_t target, int64_t v) { return (target > v) ? 1 : (target < v) ? -1 : 0; }

int64_t oracle_binary_search(const int32_t *A, int64_t lo, int64_t hi, int64_t target)
{
	int64_t s = lo, e = hi, mid;
	if (cmp_i64(target, A[s]) < 0)
		return s;
	if (cmp_i64(target, A[e]) > 0)
		return e;
	for (;;) {
		mid = (s + e) / 2;
		if (mid == s || mid == e)
			break;
		if (cmp_i64(target, A[mid]) > 0)
			s = mid;
		else
			e = mid;
	}
	if (cmp_i64(target, A[s]) == 0)
		return s;
	if (cmp_i64(target, A[e]) == 0)
		return e;
	{
		int64_t ds = target - A[s]; if (ds < 0) ds = -ds;
		int64_t de = target - A[e]; if (de < 0) de = -de;
		return (ds < de) ? s : e;
	}
}

/* ---------------------------------------------------------------------------------------------------------
 * loop_partitioner_balance_prefix_sums(W, w, row_ptr, m, nnz, &s, &e)  (parallel_util.h:141-165)
 * Worker w gets rows [s, e): s = nearest index of row_ptr[0..m-1] to nnz*w/W (worker 0 starts at 0, the last
 * worker ends at m).  Integer division exactly as the macro (total_sum * (long) w) / (long) W.
 * ------------------------------------------------------------------------------------------------------- */
void oracle_partition(const int32_t *row_ptr, int64_t m, int64_t nnz, int64_t W, int64_t w,
                      int64_t *s_out, int64_t *e_out)
{
	int64_t target = (nnz * w) / W;
	int64_t target_next = (nnz * (w + 1)) / W;
	int64_t s, e;
	if (w == 0)
		s = 0;
	else
		s = oracle_binary_search(row_ptr, 0, m - 1, target);
	if (w == W - 1)
		e = m;
	else
		e = oracle_binary_search(row_ptr, 0, m - 1, target_next);
	*s_out = s;
	*e_out = e;
}

/* ---------------------------------------------------------------------------------------------------------
 * CheckAccuracy gold (spmv_bench.cpp:130-160): per (row i, column n) a Kahan-compensated __float128 sum of
 * a_ref[j] * x_ref[n*ncols + ja[j]].  Values are widened from double (csr_a_ref and x_ref are double in the
 * harness for both the _d and _f builds, spmv_bench.cpp:121,579).
 * ------------------------------------------------------------------------------------------------------- */
void oracle_gold(const int32_t *ia, const int32_t *ja, const double *a_ref, int64_t m, int64_t ncols,
                 const double *x_ref, int32_t k, __float128 *y_gold)
{
	#pragma omp parallel for schedule(static)
	for (int64_t i = 0; i < m; i++) {
		for (int64_t n = 0; n < k; n++) {
			__float128 sum = 0, comp = 0, val, tmp;
			for (int64_t j = ia[i]; j < ia[i + 1]; j++) {
				val = (__float128) a_ref[j] * (__float128) x_ref[n * ncols + ja[j]] - comp;
				tmp = sum + val;
				comp = (tmp - sum) - val;
				sum = tmp;
			}
			y_gold[i * k + n] = sum;
		}
	}
}

/* Gold rounded to double, for callers without binary128. */
void oracle_gold_to_double(const int32_t *ia, const int32_t *ja, const double *a_ref, int64_t m, int64_t ncols,
                           const double *x_ref, int32_t k, double *y_gold_d, double *y_absdot)
{
	#pragma omp parallel for schedule(static)
	for (int64_t i = 0; i < m; i++) {
		for (int64_t n = 0; n < k; n++) {
			__float128 sum = 0, comp = 0, val, tmp;
			double absdot = 0;
			for (int64_t j = ia[i]; j < ia[i + 1]; j++) {
				double p = a_ref[j] * x_ref[n * ncols + ja[j]];
				val = (__float128) a_ref[j] * (__float128) x_ref[n * ncols + ja[j]] - comp;
				tmp = sum + val;
				comp = (tmp - sum) - val;
				sum = tmp;
				absdot += fabs(p);
			}
			y_gold_d[i * k + n] = (double) sum;
			if (y_absdot)
				y_absdot[i * k + n] = absdot;
		}
	}
}

/* ---------------------------------------------------------------------------------------------------------
 * CheckAccuracy report (spmv_bench.cpp:162-203).
 * out[0] = max relative diff over entries with y_gold > eps (signed test, :169)
 * out[1..8] = mae, max_ae, mse, mape, smape, lnQ_error, mlare, gmare (array_metrics.c definitions; A = gold,
 *             F = test, both read as double).
 * The reference computes the metrics with OpenMP reductions (partition-dependent last bits); this restatement
 * sums serially, so golden comparisons use a relative tolerance on the metric values.
 * ------------------------------------------------------------------------------------------------------- */
void oracle_check_accuracy(const __float128 *y_gold, const double *y_test, int64_t N, double eps, double *out)
{
	__float128 maxdiff = 0;
	for (int64_t i = 0; i < N; i++) {
		__float128 diff = y_gold[i] - (__float128) y_test[i];
		if (diff < 0) diff = -diff;
		if (y_gold[i] > (__float128) eps) {
			__float128 g = y_gold[i] < 0 ? -y_gold[i] : y_gold[i];
			diff = diff / g;
			if (diff > maxdiff) maxdiff = diff;
		}
	}
	double mae = 0, max_ae = 0, mse = 0, mare = 0, smare = 0, lnq = 0;
	for (int64_t i = 0; i < N; i++) {
		double a = (double) y_gold[i], f = y_test[i];
		double ae = fabs(a - f);
		mae += ae;
		if (ae > max_ae) max_ae = ae;
		mse += (a - f) * (a - f);
		mare += ae / fmax(fabs(a), DBL_EPSILON);
		smare += ae / fmax(fabs(a) + fabs(f), DBL_EPSILON);
		lnq += log10(fmax(fabs(f), DBL_EPSILON)) - log10(fmax(fabs(a), DBL_EPSILON));
	}
	double n = (double) N;
	out[0] = (double) maxdiff;
	out[1] = mae / n;
	out[2] = max_ae;
	out[3] = mse / n;
	out[4] = 100.0 * mare / n;
	out[5] = 100.0 * smare / n;
	out[6] = lnq / n;
	{
		long double e = out[6];
		out[7] = (double) log10l(fabsl(powl(10, e) - 1));
	}
	out[8] = pow(10, out[7]);
}

/* ---------------------------------------------------------------------------------------------------------
 * coo_to_csr(R, C, V, m, n, nnz, row_ptr, col_idx, values, sort_columns=1, transpose=0)  (csr_gen.c:163-217),
 * as the reference runs it with ONE OpenMP thread:
 *  - bucketsort by row (lib/sort/bucketsort/bucketsort_gen.c:163-199): counts, inclusive scan, then entry i takes
 *    slot --end[row] -- each row holds its COO entries in reverse order.  (With several threads the slots are
 *    handed out by an atomic decrement in whatever order the threads arrive: the reference's order among duplicate
 *    (row, col) entries is then not reproducible.)
 *  - csr_sort_columns (csr_gen.c:83-156) per row: degree > n/5 -> stable bucket sort by column
 *    (bucketsort_stable_serial, bucketsort_gen.c:127-160); otherwise quicksort of the entry indices keyed by column
 *    (quicksort_gen.c:93-127: partition [s, e], push s, continue right; when a part is one element, e-- and pop),
 *    partitions by partition_auto_serial (partition_gen.c:269-294: sizes 1 and 2 directly, else median of three
 *    at s, (s+e)/2, e, then partition_serial_base (:146-193) of [s+1, e-1] around the middle entry).
 * Indexing does not depend on any of this; the VALUE order among duplicates does, and is pinned against the
 * reference run with one thread (tests/golden/make_golden.py sets it).
 * ------------------------------------------------------------------------------------------------------- */
static int qs_cmp(int32_t a, int32_t b, const int32_t *key)
{
	return (key[a] > key[b]) ? 1 : (key[a] < key[b]) ? -1 : 0;
}

static int64_t qs_partition_base(int32_t pivot, int32_t *A, int64_t lo, int64_t hi, const int32_t *key)
{
	while (1) {
		while (lo < hi && qs_cmp(A[lo], pivot, key) < 0) lo++;
		while (lo < hi && qs_cmp(A[hi], pivot, key) > 0) hi--;
		if (lo >= hi) break;
		int32_t t = A[lo]; A[lo] = A[hi]; A[hi] = t;
		lo++; hi--;
	}
	if (qs_cmp(A[lo], pivot, key) < 0) lo++;
	return lo;
}

#define QS_SWAP(x, y) do { int32_t _t = (x); (x) = (y); (y) = _t; } while (0)

static int64_t qs_partition_auto(int32_t *A, int64_t s, int64_t e_excl, const int32_t *key)
{
	if (e_excl - s == 1) return s;
	if (e_excl - s == 2) {
		if (qs_cmp(A[s], A[s + 1], key) > 0) QS_SWAP(A[s], A[s + 1]);
		return s + 1;
	}
	int64_t e = e_excl - 1, p = (s + e) / 2;
	if (qs_cmp(A[s], A[e], key) > 0) QS_SWAP(A[s], A[e]);
	if (qs_cmp(A[s], A[p], key) > 0) QS_SWAP(A[s], A[p]);
	if (qs_cmp(A[p], A[e], key) > 0) QS_SWAP(A[p], A[e]);
	return qs_partition_base(A[p], A, s + 1, e - 1, key);
}

static void qs_sort(int32_t *A, int64_t N, const int32_t *key, int64_t *parts)
{
	if (N < 2) return;
	int64_t s = 0, e = N - 1, i = 0;
	while (1) {
		while (s >= e) {
			if (s == 0) return;
			i--;
			e--;
			s = parts[i];
		}
		int64_t mid = qs_partition_auto(A, s, e + 1, key);
		parts[i++] = s;
		s = mid;
	}
}

void oracle_coo_to_csr(const int32_t *R, const int32_t *C, const double *V, int64_t m, int64_t n, int64_t nnz,
                       int32_t *row_ptr, int32_t *col_idx, double *values)
{
	int64_t *end = (int64_t *) calloc(m + 1, sizeof(int64_t));
	int32_t *Cb = (int32_t *) malloc((nnz > 0 ? nnz : 1) * sizeof(int32_t));
	double *Vb = (double *) malloc((nnz > 0 ? nnz : 1) * sizeof(double));
	int32_t *perm = (int32_t *) malloc((nnz > 0 ? nnz : 1) * sizeof(int32_t));
	int64_t *parts = (int64_t *) malloc((nnz + 1) * sizeof(int64_t));
	int64_t *cnt = (int64_t *) calloc((n > 0 ? n : 1) + 1, sizeof(int64_t));
	for (int64_t i = 0; i < nnz; i++) end[R[i] + 1]++;
	for (int64_t i = 0; i < m; i++) end[i + 1] += end[i];
	for (int64_t i = 0; i <= m; i++) row_ptr[i] = (int32_t) end[i];
	for (int64_t i = 0; i < nnz; i++) {                 /* one thread: slots handed out from each row's end */
		int64_t p = --end[R[i] + 1];
		Cb[p] = C[i];
		Vb[p] = V ? V[i] : 1.0;
	}
	for (int64_t i = 0; i < m; i++) {
		int64_t s = row_ptr[i], deg = row_ptr[i + 1] - s;
		if (deg == 0) continue;
		if (deg > n / 5) {                               /* stable bucket sort by column */
			for (int64_t q = 0; q < deg; q++) cnt[Cb[s + q] + 1]++;
			for (int64_t c = 0; c < n; c++) cnt[c + 1] += cnt[c];
			for (int64_t q = 0; q < deg; q++) perm[cnt[Cb[s + q]]++] = (int32_t) q;
			memset(cnt, 0, ((n > 0 ? n : 1) + 1) * sizeof(int64_t));
		} else {
			for (int64_t q = 0; q < deg; q++) perm[q] = (int32_t) q;
			qs_sort(perm, deg, Cb + s, parts);
		}
		for (int64_t q = 0; q < deg; q++) {
			col_idx[s + q] = Cb[s + perm[q]];
			if (values) values[s + q] = Vb[s + perm[q]];
		}
	}
	free(end); free(Cb); free(Vb); free(perm); free(parts); free(cnt);
}

/* drand48 stream (POSIX: X_{n+1} = (0x5DEECE66D X_n + 0xB) mod 2^48, srand48(s): X = s<<16 | 0x330E), used
 * for the seeded-B golden inputs (benchmark_code/GPU/NVIDIA-CUDA/spmv_code_cusparse-11.x/src/spmv_utils.cpp:236-249
 * seeds x with srand48(42)). */
void oracle_drand48_fill(int64_t seed, double *out, int64_t n)
{
	uint64_t X = (((uint64_t) seed) << 16) | 0x330EULL;
	for (int64_t i = 0; i < n; i++) {
		X = (0x5DEECE66DULL * X + 0xBULL) & ((1ULL << 48) - 1);
		out[i] = ldexp((double) X, -48);
	}
}


/* ---------------------------------------------------------------------------------------------------------
 * Pipeline SDDMM  (pipeline_code_bench/sddmm_taco_naive.cpp:98-140, 280-290)
 *   compute_csr zeroes y, then compute2 adds, for every mask nonzero pA2 of row mA, O[mA][nD] * D[mA][nD] over nD
 *   (O = Q, D = K, both [m][n] row-major; kA = the nonzero's column is read but not used: row mA of K), then
 *   multiplies by the mask value.  `B += O*D` is contracted to fma by the reference flags.  mode 1 restates the
 *   attention SDDMM the pipeline intends (row kA = col of the nonzero), same chain order.
 * ------------------------------------------------------------------------------------------------------- */
void oracle_sddmm_d(const int32_t *ia, const int32_t *ja, const double *a, int64_t m, const double *Q,
                    const double *K, int32_t n, int32_t mode, double *y)
{
	for (int64_t i = 0; i < m; i++)
		for (int64_t p = ia[i]; p < ia[i + 1]; p++) {
			const int64_t kr = mode ? ja[p] : i;
			double acc = 0;
			for (int64_t t = 0; t < n; t++)
				acc = fma(Q[i * n + t], K[kr * n + t], acc);
			y[p] = acc * a[p];
		}
}

void oracle_sddmm_f(const int32_t *ia, const int32_t *ja, const float *a, int64_t m, const float *Q,
                    const float *K, int32_t n, int32_t mode, float *y)
{
	for (int64_t i = 0; i < m; i++)
		for (int64_t p = ia[i]; p < ia[i + 1]; p++) {
			const int64_t kr = mode ? ja[p] : i;
			float acc = 0;
			for (int64_t t = 0; t < n; t++)
				acc = fmaf(Q[i * n + t], K[kr * n + t], acc);
			y[p] = acc * a[p];
		}
}

/* softmax over all nonzeros, serial (sddmm_taco_naive.cpp:191-209) */
void oracle_softmax_d(double *y, int64_t nnz)
{
	if (nnz <= 0) return;
	double mx = y[0], sum = 0;
	for (int64_t i = 1; i < nnz; i++) if (y[i] > mx) mx = y[i];
	for (int64_t i = 0; i < nnz; i++) { y[i] = exp(y[i] - mx); sum += y[i]; }
	for (int64_t i = 0; i < nnz; i++) y[i] /= sum;
}

void oracle_softmax_f(float *y, int64_t nnz)
{
	if (nnz <= 0) return;
	float mx = y[0], sum = 0;
	for (int64_t i = 1; i < nnz; i++) if (y[i] > mx) mx = y[i];
	for (int64_t i = 0; i < nnz; i++) { y[i] = expf(y[i] - mx); sum += y[i]; }
	for (int64_t i = 0; i < nnz; i++) y[i] /= sum;
}

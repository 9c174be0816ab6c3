"""The wide-window policy on the host (spmm_hip_debug_plan, no GPU): fp64 K = 32 matrices of >= 2.5 M
nonzeros whose rows average >= 256 plan blocks of up to 4,096 nonzeros; smaller or shorter-row matrices, fp32, other
K, and plans that take column windows keep the 2,048-nonzero window."""
import spmm_amd as S


def cap(line, k=32, dtype=S.F64, env=None, monkeypatch=None):
    A = S.generate(S.gen_params(line))
    return int(S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, dtype)["cap"])


def test_wide_window_policy(monkeypatch):
    for v in ("SPMM_HIP_CAP", "SPMM_HIP_MFMA", "SPMM_HIP_TILES"):
        monkeypatch.delenv(v, raising=False)
    big500 = "5588 5588 500 166.6667 normal random 0.3 1000 1.9 0.5 14"
    assert cap(big500) == 4096
    assert cap(big500, k=8) == 2048                     # 64-B rows: groups of 4 lanes, no wide kernel
    assert cap(big500, k=128) == 2048                   # measured at K = 32 only
    assert cap(big500, dtype=S.F32) == 2048
    assert cap("4191 4191 500 166.6667 normal random 0.3 0 0.05 0.05 14") == 2048     # < 2.5 M nonzeros
    assert cap("27869 27869 100 33.3333 normal random 0.6 0 0.5 0.05 14") == 2048     # rows of 100
    monkeypatch.setenv("SPMM_HIP_CAP", "2048")
    assert cap(big500) == 2048                          # the A/B's off switch

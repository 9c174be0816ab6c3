#!/usr/bin/env python3
"""tools/pair_census.py -- the paired-rows policy decision (spmm_hip_debug_plan, host only) per generator line of a
line file at fp64 K 8 / 32 and fp32 K 32: {"gen", "<dtype>_k<K>": [pair, sampled reuse]}.  Note: the census in
profiles/r06/pair/ was taken before the fp64-only and 4 M-nonzero floor were added."""
import json, sys
import spmm_amd as S
for line in open(sys.argv[1]).read().split('\n'):
    if not line.strip(): continue
    A = S.generate(S.gen_params(line))
    out = {"gen": line}
    for k, dt in ((8, S.F64), (32, S.F64), (32, S.F32)):
        p = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, dt)
        out[f"{'f64' if dt == S.F64 else 'f32'}_k{k}"] = [int(p["pair"]), round(p["pair_reuse"], 3)]
    print(json.dumps(out), flush=True)

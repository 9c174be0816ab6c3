#!/usr/bin/env python3
"""tools/gate_rules.py -- round-5 gate fit per value type on the A/B records of profiles/r05/fit/ (fit_mfma_gate.py's
model, the B range-check term included), then the outcome of candidate rules (tile share, model gain, the K < 64
rows rule) per (K, avg, crs) class: pairs taken, worst and median speedup.  Writes profiles/r05/fit/gate_fit.json.

  python tools/gate_rules.py
"""
import sys, json, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import fit_mfma_gate as fm
from collections import defaultdict
from scipy.optimize import least_squares
res={}
for dt, feat in (("f64", ROOT / "profiles/r04/fit_features.jsonl"), ("f32", ROOT / "profiles/r05/fit/fit_features_f32.jsonl")):
    ab=fm.load_ab([str(ROOT / "profiles/r05/fit/fit_ab.w*.jsonl")], dt)
    feats={}
    for l in open(feat):
        d=json.loads(l)
        if d.get("dtype","f64")==dt: feats[(d["gen"],d["k"])]=d
    keys=[k for k in ab if k in feats and ab[k]["tile_mode"]=="mfma"]
    F={f: np.array([feats[k][f] if f in feats[k] else ab[k][f] for k in keys], float) for f in ("k","nnz","m","est_chunks","est_tiles","est_tile_nnz","max_chunks","r16","kw")}
    F["vsize"]=np.full(len(keys), 8.0 if dt=="f64" else 4.0)
    t_on=np.array([ab[k]["ms"]*1e3 for k in keys]); t_off=np.array([ab[k]["ms_base"]*1e3 for k in keys])
    base={"min_tile_frac":0.0,"gain":1.0}
    def c_of(x,y): return {**base,"launch":y[0],"row_us_nnz":y[1],"row_reuse_exp":y[2],"row_kw_exp":y[3],"row_us_row":y[4],"mfma_launch":x[0],"us_chunk":x[1],"us_tile":x[2],"us_chain":x[3],"us_bmb":x[4]}
    y=least_squares(lambda y: np.log(fm.model(F,c_of([0,0,0,0,0],y))[1]/t_off),[5,2.5e-5,0.2,0.15,1e-4],bounds=([0,0,-2,-2,0],[100,1e-3,3,3,1e-2])).x
    sel=F["est_tile_nnz"]>=0.9*F["nnz"]; Fs={k:v[sel] for k,v in F.items()}
    x=least_squares(lambda x: np.log(fm.model(Fs,c_of(x,y))[0]/t_on[sel]),[20,1.6e-3,1.5e-3,1.1,0.2],bounds=([0,0,0,0,0],[200,1e-2,1e-2,50,5]),loss="soft_l1").x
    c=c_of(x,y); res[dt]=c
    print(dt, {k:(float('%.4g'%v)) for k,v in c.items()})
    for frac,gain,k32 in ((0.9,1.2,0.0),(0.9,1.2,32.0),(0.9,1.3,32.0),(0.9,1.15,32.0)):
        cc={**c,"min_tile_frac":frac,"gain":gain,"k32_min_row_nnz":k32}
        on=fm.decide(F,cc); sp=t_off/t_on
        cls=defaultdict(list)
        for i,k in enumerate(keys):
            if on[i]: cls[(k[1],int(k[0].split()[2]),k[0].split()[9])].append(sp[i])
        print(f'  frac {frac} gain {gain} k32 {k32}: taken',int(on.sum()),'worst',round(float(sp[on].min()),3) if on.any() else None,'agg',round(float(t_off.sum()/np.where(on,t_on,t_off).sum()),4))
        print('    ', {f"{a}/{b}/{cr}":(len(v),round(min(v),2),round(float(np.median(v)),2)) for (a,b,cr),v in sorted(cls.items())})
json.dump(res, open(ROOT / 'profiles/r05/fit/gate_fit.json', 'w'))

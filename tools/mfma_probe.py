#!/usr/bin/env python3
"""tools/mfma_probe.py -- measurement of the matrix-core tile kernel (spmm_mfma_tile_kernel) before it is
wired into the engine: tile tables from the engine's own inspector (spmm_hip_debug_tiles), the kernel through
lib/libmfma_probe.so, checked against the engine (tiles off) within 1e-10 normwise on every tile row, timed with HIP
events against the engine with tiles off / by policy / forced onto the same tile plan.  One JSON line per case.

  python tools/mfma_probe.py [--lines 'l1;l2'] [--rmax 32,64] [--reuse 2,4,8] [--k 32]
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))

LINES = ["39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14",
         "22354 22354 500 166.6667 normal random 0.05 100 0.05 0.05 14",
         "39120 39120 500 166.6667 normal random 0.3 0 0.5 0.95 14",
         "22354 22354 500 166.6667 normal random 0.6 100 0.95 0.95 14",
         "111476 111476 100 33.3333 normal random 0.05 100 0.05 0.5 14",
         "111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14",
         "195083 195083 100 33.3333 normal random 0.6 0 0.95 0.5 14",
         "222214 222214 50 16.6667 normal random 0.05 100 0.95 0.95 14",
         "388875 388875 50 16.6667 normal random 0.3 0 0.05 0.5 14",
         "550072 550072 20 6.6667 normal random 0.6 1000 0.5 0.95 14",
         "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"]
UC, CAPA, DMAX = 48, 512, 63


def mfma_tables(A, plan, rmax):
    """Kernel tables from the inspector's tile plan: panel cells (row * 49 + chunk column, padding -> trash), values,
    and the union columns of every chunk transposed to [g][k step] with 48 slots per chunk (padded with a valid row)."""
    pst = UC + 1
    trash = rmax * pst
    tiles, chunks, perm, tlidx, tcol = plan["tiles"], plan["chunks"], plan["perm"], plan["tlidx"], plan["tcol"]
    nz = len(perm)
    nch = len(chunks) - 1
    chunk_of = np.repeat(np.arange(nch), np.diff(chunks[:, 2]))
    tile_of_chunk = np.repeat(np.arange(len(tiles)), tiles[:, 3])
    assert len(chunk_of) == nz and len(tile_of_chunk) == nch
    row_of_nnz = np.repeat(np.arange(A.m, dtype=np.int64), np.diff(A.row_ptr.astype(np.int64)))
    real = perm >= 0
    pos = np.full(nz, trash, np.uint16)
    first_row = tiles[tile_of_chunk[chunk_of[real]], 0].astype(np.int64)
    q = row_of_nnz[perm[real]] - first_row
    assert (q >= 0).all() and (q < rmax).all() and (tlidx[real] < UC).all()
    pos[real] = (q * pst + tlidx[real]).astype(np.uint16)
    val = np.zeros(nz, np.float64)
    val[real] = A.values[perm[real]]
    # union column u (0..47) of chunk c -> slot c*48 + (u % 4) * 12 + u // 4; past U: the chunk's first column
    u = np.arange(UC)
    slot = (u % 4) * (UC // 4) + u // 4
    first = chunks[:-1, 0].astype(np.int64)
    ncl = chunks[:-1, 1].astype(np.int64)
    src = first[:, None] + np.minimum(u[None, :], ncl[:, None] - 1)
    tcolT = np.empty((nch, UC), np.int32)
    tcolT[:, slot] = tcol[src]
    return pos, val, tcolT.reshape(-1)


def has_duplicates(A):
    c = A.col_idx.astype(np.int64)
    same = c[1:] == c[:-1]
    starts = np.zeros(len(c), bool)
    starts[A.row_ptr[:-1][A.row_ptr[:-1] < len(c)]] = True
    return bool((same & ~starts[1:]).any())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", default="")
    ap.add_argument("--rmax", default="16")
    ap.add_argument("--reuse", default="2,4,8")
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--xcd", type=int, default=1)
    ap.add_argument("--dbg", default="", help="extra kernel variants timed (probe codes: 3 no MFMA, 5 no B loads)")
    ap.add_argument("--lr-lib", default="", help="also time (and check bit for bit) this probe library on the same "
                    "tables, e.g. spmm-research_amd/lib/libmfma_probe_lr.so (tools/mfma_lr.hpp)")
    ap.add_argument("--no-forced", action="store_true", help="skip the engine forced onto the tile plan")
    ap.add_argument("--variants", default="", help="with --lr-lib: also time these variants of it over all K columns, "
                    "e.g. np1r12,np1r6,np2r12,np2r6 (np 32-column sub-panels per wave, r B-operand ring slots)")
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    L = C.CDLL(str(ROOT / "spmm-research_amd" / "lib" / "libmfma_probe.so"))
    L.mfma_probe_launch.argtypes = [C.c_int] + [C.c_void_p] * 6 + [C.c_longlong, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    LR = None
    if args.lr_lib:
        LR = C.CDLL(str(ROOT / args.lr_lib))
        LR.mfma_probe_launch.argtypes = L.mfma_probe_launch.argtypes
        LR.mfma_probe_launch_v.argtypes = [C.c_int] + [C.c_void_p] * 6 + [C.c_longlong, C.c_void_p, C.c_int, C.c_int,
                                                                           C.c_int, C.c_void_p]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    k = args.k
    assert k == 32 or args.no_forced, "probe: one 32-column panel (K > 32 only with --no-forced)"
    assert k % 32 == 0

    def timed(fn):
        ts = []
        for _ in range(args.rounds):
            fn(), fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / args.iters)
        return min(ts)

    lines = args.lines.split(";") if args.lines else LINES
    for line in lines:
        A = S.generate(S.gen_params(line))
        if has_duplicates(A):
            print(json.dumps({"gen": line, "skip": "duplicate columns"}), flush=True)
            continue
        g = torch.Generator(device=dev)
        g.manual_seed(42)
        B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64) * 2 - 1
        handles = {}
        for name, env in (("off", {"SPMM_HIP_TILES": "-1"}), ("policy", {})):
            for kk, vv in env.items():
                os.environ[kk] = vv
            handles[name] = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
            for kk in env:
                os.environ.pop(kk)
        absh = S.csr_to_format(A.row_ptr, A.col_idx, np.abs(A.values), A.m, A.ncols, A.nnz, k, 0)
        C_ref = torch.empty((A.m, k), device=dev, dtype=torch.float64)
        C_abs = torch.empty_like(C_ref)
        handles["off"].spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C_ref.data_ptr(), k, sp)
        Babs = B.abs()
        absh.spmm_device(Babs.data_ptr(), S.B_ROW_MAJOR, C_abs.data_ptr(), k, sp)
        torch.cuda.synchronize()
        absh.close()
        Cx = torch.empty_like(C_ref)
        t_off = timed(lambda: handles["off"].spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cx.data_ptr(), k, sp))
        t_pol = timed(lambda: handles["policy"].spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cx.data_ptr(), k, sp))
        T = handles["off"].seq_max
        out = {"gen": line, "nnz": A.nnz, "m": A.m, "T": T, "off_ms": round(t_off, 5), "policy_ms": round(t_pol, 5),
               "policy_tiles": handles["policy"].tile_info()["tiles"], "cases": []}
        for rmax in (int(x) for x in args.rmax.split(",")):
            for reuse in (float(x) for x in args.reuse.split(",")):
                plan = S.debug_tiles(A.row_ptr, A.col_idx, A.ncols, T, rmax=rmax, uc=UC, capa=CAPA,
                                     min_reuse=reuse, colmax=DMAX * UC - 4, dmax=DMAX)
                nt = len(plan["tiles"])
                case = {"rmax": rmax, "reuse": reuse, "tiles": nt}
                if nt == 0:
                    out["cases"].append(case)
                    continue
                pos, val, tcolT = mfma_tables(A, plan, rmax)
                d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                d_tiles = d(plan["tiles"].astype(np.int32))
                d_chunks = d(plan["chunks"].astype(np.int32))
                d_tcol = d(tcolT)
                d_val = d(np.concatenate([val, np.zeros(8)]))
                d_pos = d(np.concatenate([pos, np.zeros(8, np.uint16)]).view(np.int16))
                Cm = torch.zeros_like(C_ref)
                bb = A.ncols * k * 8
                def launch(xcd=args.xcd, lib=L, Cout=None):      # the kernel over every 32-column sub-panel
                    Co = Cm if Cout is None else Cout
                    r = 0
                    for k1 in range(0, k, 32):
                        r |= lib.mfma_probe_launch(nt, d_tiles.data_ptr(), d_chunks.data_ptr(), d_tcol.data_ptr(),
                                                   d_val.data_ptr(), d_pos.data_ptr(), B.data_ptr() + 8 * k1,
                                                   bb - 8 * k1, Co.data_ptr() + 8 * k1, k, xcd, sp)
                    return r
                st = launch()
                torch.cuda.synchronize()
                assert st == 0, st
                rows = torch.from_numpy(plan["in_tile"]).to(dev)
                err = (Cm[rows] - C_ref[rows]).abs()
                tol = 1e-10 * torch.maximum(C_ref[rows].abs(), C_abs[rows]) + 1e-300
                ok = bool((err <= tol).all().item())
                case["max_err_over_absdot"] = float((err / (C_abs[rows] + 1e-300)).max().item())
                case["ok"] = ok
                ex = rows & torch.from_numpy(handles["off"].exact_rows()).to(dev)
                case["bitexact_rows"] = int(ex.sum().item())
                case["bitexact"] = bool(torch.equal(Cm[ex].view(torch.int64), C_ref[ex].view(torch.int64)))
                t_m = timed(launch)
                for v in (int(x) for x in args.dbg.split(",") if x):
                    case[f"dbg{v}_ms"] = round(timed(lambda: launch(v)), 5)
                if LR is not None:
                    Cl = torch.zeros_like(C_ref)
                    lr = lambda: launch(lib=LR, Cout=Cl)
                    assert lr() == 0
                    torch.cuda.synchronize()
                    case["lr_same_as_mfma"] = bool(torch.equal(Cl[rows].view(torch.int64), Cm[rows].view(torch.int64)))
                    case["lr_bitexact"] = bool(torch.equal(Cl[ex].view(torch.int64), C_ref[ex].view(torch.int64)))
                    case["lr_ms"] = round(timed(lr), 5)
                    for v in (x for x in args.variants.split(",") if x):
                        npv, rv = int(v[2]), int(v.split("r")[1])
                        Cl.zero_()
                        fv = lambda: LR.mfma_probe_launch_v(nt, d_tiles.data_ptr(), d_chunks.data_ptr(),
                                                            d_tcol.data_ptr(), d_val.data_ptr(), d_pos.data_ptr(),
                                                            B.data_ptr(), bb, Cl.data_ptr(), k, npv, rv, sp)
                        assert fv() == 0
                        torch.cuda.synchronize()
                        case[f"{v}_same"] = bool(torch.equal(Cl[rows].view(torch.int64), Cm[rows].view(torch.int64)))
                        case[f"{v}_ms"] = round(timed(fv), 5)
                    del Cl
                if args.no_forced:
                    tile_nnz = int(np.diff(A.row_ptr)[plan["in_tile"]].sum())
                    case.update({"tile_nnz": tile_nnz, "chunks": int(len(plan["chunks"]) - 1), "mfma_ms": round(t_m, 5)})
                    out["cases"].append(case)
                    del d_tiles, d_chunks, d_tcol, d_val, d_pos, Cm
                    continue
                os.environ.update({"SPMM_HIP_TILES": "1", "SPMM_HIP_TILE_REUSE": str(reuse),
                                   "SPMM_HIP_TILE_ROWS": str(rmax)})
                hf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
                for kk in ("SPMM_HIP_TILES", "SPMM_HIP_TILE_REUSE", "SPMM_HIP_TILE_ROWS"):
                    os.environ.pop(kk)
                t_f = timed(lambda: hf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cx.data_ptr(), k, sp))
                ti = hf.tile_info()
                hf.close()
                tile_nnz = int(np.diff(A.row_ptr)[plan["in_tile"]].sum())
                case.update({"tile_rows": int(plan["in_tile"].sum()), "tile_nnz": tile_nnz,
                             "chunks": int(len(plan["chunks"]) - 1), "density": round(tile_nnz / max(1, (len(plan["chunks"]) - 1)) / (rmax * UC), 4),
                             "mfma_ms": round(t_m, 5), "forced_ms": round(t_f, 5), "forced_tiles": ti["tiles"],
                             "mfma_tile_tflops": round(2 * tile_nnz * k / t_m / 1e9, 2)})
                out["cases"].append(case)
                del d_tiles, d_chunks, d_tcol, d_val, d_pos, Cm
        print(json.dumps(out), flush=True)
        for h in handles.values():
            h.close()
        del B, Babs, C_ref, C_abs, Cx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

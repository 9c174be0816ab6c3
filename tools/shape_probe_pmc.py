#!/usr/bin/env python3
"""tools/shape_probe_pmc.py -- the counters of tools/shape_probe.py's kernels, per line and kernel (verdict r05 item 1).

Reads a session directory with the kernel trace (kt/) and the PMC passes (pa/ pb/ pc/ pd/ of tools/sessions/r06_b.sh),
attributes every dispatch to its generator line by order (each line runs: the engine twice, then flat, then the
three rows probes), averages each counter per (line, kernel), and prints one markdown table per line:

  us          mean kernel duration (kernel trace)
  occupancy   SQ_WAVE_CYCLES / SQ_BUSY_CYCLES x 4: mean resident waves per CU (SQ counts per SIMD... see note)
  vmem/wave   SQ_INST_LEVEL_VMEM / SQ_WAVE_CYCLES: vector-memory instructions in flight per resident wave
  wait        SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier); issue = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  TA busy     TA_TA_BUSY_sum / (256 x GRBM_GUI_ACTIVE / 8): fraction of kernel cycles a CU's texture addresser is busy
  L2 req      TCP_TCC_READ_REQ_sum per launch; L2 lat = TCP_TCC_READ_REQ_LATENCY_sum / TCP_TCC_READ_REQ_sum (cycles)
  L2 hit      TCC_HIT / (TCC_HIT + TCC_MISS); past-L2 = 2 x FETCH_SIZE KiB (gfx950 correction)
  VMEM/LDS/VALU instructions per nonzero (SQ_INSTS_*; wave instructions)

  python tools/shape_probe_pmc.py gpurun_out/r06b [--nnz n1,n2,...]
"""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path

KINDS = [("spmm_rows_kernel", "engine"), ("flat_probe", "flat"), ("rows_probe<16, 2048, false>", "rows_gather"),
         ("rows_probe<16, 2048, true>", "rows_fma"), ("rows_probe<16, 8192, true>", "rows_fma_8k")]


def kind_of(name: str):
    for key, k in KINDS:
        if key in name:
            return k
    return None


def attribute(rows, key_id="Dispatch_Id"):
    """[(line index, kind, row)] in dispatch order: a new line starts at the first engine dispatch after a probe."""
    out = []
    line = -1
    prev = None
    for r in sorted(rows, key=lambda r: int(r[key_id])):
        k = kind_of(r["Kernel_Name"])
        if k is None:
            continue
        if k == "engine" and prev not in (None, "engine"):
            line += 1
        if line < 0:
            line = 0
        out.append((line, k, r))
        prev = k
    return out


def load_pmc(d: Path):
    """{(line, kind): {counter: mean per dispatch}}"""
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(d.rglob("*counter_collection.csv")):
        rows = list(csv.DictReader(open(f)))
        # one row per (dispatch, counter): collapse to dispatches first
        disp = {}
        for r in rows:
            dd = disp.setdefault(r["Dispatch_Id"], {"Dispatch_Id": r["Dispatch_Id"], "Kernel_Name": r["Kernel_Name"],
                                                    "c": defaultdict(float)})
            dd["c"][r["Counter_Name"]] += float(r["Counter_Value"])
        for line, k, r in attribute(list(disp.values())):
            for c, v in r["c"].items():
                vals[(line, k)][c].append(v)
    return {key: {c: sum(v) / len(v) for c, v in cs.items()} for key, cs in vals.items()}


def load_durations(d: Path):
    f = next(d.rglob("*kernel_trace.csv"))
    dur = defaultdict(list)
    for line, k, r in attribute(list(csv.DictReader(open(f)))):
        dur[(line, k)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {key: sorted(v)[len(v) // 2] for key, v in dur.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--probe", default=None, help="probe.jsonl of the session (nnz per line, labels)")
    args = ap.parse_args()
    d = Path(args.dir)
    probe = [json.loads(l) for l in open(args.probe or d / "probe.jsonl")]
    dur = load_durations(d / "kt")
    pmc = {}
    for p in ("pa", "pb", "pc", "pd"):
        if (d / p).exists():
            for key, cs in load_pmc(d / p).items():
                pmc.setdefault(key, {}).update(cs)
    out = []
    for li, rec in enumerate(probe):
        nnz = rec["nnz"]
        out.append(f"\n#### {rec['gen']} (nnz {nnz / 1e6:.2f} M, B {rec['b_mb']:.1f} MB, K = 32 fp64)\n")
        out.append("| kernel | us | B rows TB/s | waves/CU | vmem in flight/wave | wait | issue stall | TA busy | "
                   "L2 req/nnz | L2 lat (cyc) | L2 hit | past-L2 MB | VMEM/nnz | LDS/nnz | VALU/nnz |")
        out.append("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
        for _, k in KINDS:
            c = pmc.get((li, k), {})
            t = dur.get((li, k))
            if t is None:
                continue
            g = lambda n: c.get(n)  # noqa

            def ratio(a, b, scale=1.0):
                return None if g(a) is None or not g(b) else g(a) / g(b) * scale
            gui = g("GRBM_GUI_ACTIVE")
            ta = None if g("TA_TA_BUSY_sum") is None or not gui else g("TA_TA_BUSY_sum") / (256 * gui / 8)
            # SQ_BUSY_CYCLES / SQ_WAVE_CYCLES are summed over the chip's SQs; waves per CU = wave-cycles / busy cycles
            # per CU (busy counted per SE: 32 SEs, 8 CUs each)
            occ = None if g("SQ_WAVE_CYCLES") is None or not g("SQ_BUSY_CYCLES") else \
                g("SQ_WAVE_CYCLES") / g("SQ_BUSY_CYCLES") / 8
            hit = None
            if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
                hit = g("TCC_HIT_sum") / max(g("TCC_HIT_sum") + g("TCC_MISS_sum"), 1)
            fetch = None if g("FETCH_SIZE") is None else 2 * g("FETCH_SIZE") * 1024 / 1e6
            row = [k, f"{t:.1f}", f"{nnz * 256 / (t * 1e-6) / 1e12:.1f}",
                   occ, ratio("SQ_INST_LEVEL_VMEM", "SQ_WAVE_CYCLES"), ratio("SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
                   ratio("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"), ta,
                   None if g("TCP_TCC_READ_REQ_sum") is None else g("TCP_TCC_READ_REQ_sum") / nnz,
                   ratio("TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum"), hit, fetch,
                   None if g("SQ_INSTS_VMEM_RD") is None else g("SQ_INSTS_VMEM_RD") / nnz,
                   None if g("SQ_INSTS_LDS") is None else g("SQ_INSTS_LDS") / nnz,
                   None if g("SQ_INSTS_VALU") is None else g("SQ_INSTS_VALU") / nnz]
            out.append("| " + " | ".join(x if isinstance(x, str) else "—" if x is None else f"{x:.3g}" for x in row)
                       + " |")
    text = "\n".join(out)
    print(text)


if __name__ == "__main__":
    main()

"""Per-kernel PMC summary of tools/profile_model_pmc.sh passes over tools/pmc_model.py -> pmc_mfma.json.

    python tools/pmc_model_summary.py OUTDIR --model M --batch B --depth D --iters I --round rNN

Each pass directory under OUTDIR holds rocprofv3's *counter_collection.csv (and *kernel_trace.csv).
The profiled forwards are the LAST dispatches of each hot kernel (pmc_model.py runs nothing after
them): per forward fc1 and the fused qkv+attention D times, LayerNorm and the residual GEMM 2D times
(proj and fc2 alternate, proj first). Per kernel and counter: the median over those dispatches.

Conventions (MI355X_MICROARCH.md): GRBM_GUI_ACTIVE is summed over the 8 XCDs (effective clock =
GUI_ACTIVE / 8 / duration); SQ_VALU_MFMA_BUSY_CYCLES counts the matrix pipe's busy cycles summed over
every SIMD, so the busy fraction = MFMA_BUSY / (GUI_ACTIVE / 8 x CUs x 4); FETCH_SIZE is doubled
(gfx950 tallies 128-B requests at 64 B), WRITE_SIZE is taken as is; both are KB.
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics

ROLES = {
    "fc1": (re.compile(r"gemm_kernel<4, 2, 1(, (true|false|\d))?(, (true|false))?>"), 1),
    "resid": (re.compile(r"gemm_kernel<4, 1, 1(, (true|false|\d))?(, (true|false))?>"), 2),
    "qkv_attn": (re.compile(r"qkv_attn_kernel<"), 1),
    "ln": (re.compile(r"layernorm_quant_persist_kernel<"), 2),
}
CUS = 256


def rows_of(d):
    pmc, trace = [], {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        pmc += list(csv.DictReader(open(f)))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            trace[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return pmc, trace


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--model", default="vit_base_patch16_224")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--round", default="r02")
    ap.add_argument("--dest", default="")
    a = ap.parse_args()

    vals = {}   # role -> counter -> [values]
    durs = {}   # role -> [ns]
    for d in sorted(glob.glob(os.path.join(a.out, "p*"))):
        if not os.path.isdir(d):
            continue
        pmc, trace = rows_of(d)
        for role, (pat, mult) in ROLES.items():
            want = a.iters * a.depth * mult
            by_disp = {}
            for r in pmc:
                if pat.search(r.get("Kernel_Name", "")):
                    by_disp.setdefault(int(r["Dispatch_Id"]), []).append(r)
            ids = sorted(by_disp)[-want:]
            if not ids:
                continue
            names = [role] if role != "resid" else ["proj", "fc2"]
            for i, di in enumerate(ids):
                name = names[i % len(names)]
                for r in by_disp[di]:
                    vals.setdefault(name, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                if str(di) in trace:
                    durs.setdefault(name, []).append(trace[str(di)])

    kernels = {}
    for name, cs in vals.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        k = {"counters_median": med, "dispatches": max(len(v) for v in cs.values())}
        g = med.get
        if durs.get(name):
            k["duration_us_profiled"] = statistics.median(durs[name]) / 1e3
        if g("GRBM_GUI_ACTIVE"):
            cyc = g("GRBM_GUI_ACTIVE") / 8
            if g("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
                k["mfma_busy_frac"] = g("SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * CUS * 4)
            if k.get("duration_us_profiled"):
                k["clock_GHz"] = cyc / (k["duration_us_profiled"] * 1e3)
                if g("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
                    # the same busy cycles against the nominal 2.4 GHz peak over the kernel's duration
                    k["mfma_busy_frac_at_2p4GHz"] = g("SQ_VALU_MFMA_BUSY_CYCLES") / (
                        k["duration_us_profiled"] * 1e3 * 2.4 * CUS * 4)
        if g("FETCH_SIZE") is not None:
            k["fetch_bytes"] = 2.0 * g("FETCH_SIZE") * 1024
        if g("WRITE_SIZE") is not None:
            k["write_bytes"] = g("WRITE_SIZE") * 1024
        if "fetch_bytes" in k and "write_bytes" in k:
            k["traffic_bytes"] = k["fetch_bytes"] + k["write_bytes"]
        if g("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if g(c) is not None:
                    k[c.lower() + "_frac"] = g(c) / g("SQ_WAVE_CYCLES")
        if g("SQ_LDS_IDX_ACTIVE") and g("SQ_LDS_BANK_CONFLICT") is not None:
            k["lds_conflict_share"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")
        kernels[name] = k

    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from kstats import _build_id
    out = {"model": a.model, "batch": a.batch, "round": a.round, "lib_build_id": _build_id(),
           "source": "tools/profile_model_pmc.sh (rocprofv3 --pmc, one counter group per run, kernel-trace only) "
                     "over tools/pmc_model.py",
           "conventions": __doc__.split("Conventions (MI355X_MICROARCH.md): ")[1].strip(),
           "kernels": kernels}
    dests = [a.out] + ([a.dest] if a.dest else [])
    for d in dests:
        os.makedirs(d, exist_ok=True)
        for n in (f"pmc_mfma_{a.round}.json", "pmc_mfma.json"):
            with open(os.path.join(d, n), "w") as fh:
                json.dump(out, fh, indent=1)
    for name, k in kernels.items():
        print(name, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in k.items() if x != "counters_median"})


if __name__ == "__main__":
    main()

"""rocprofv3 summaries.

    python tools/kstats.py STATS_CSV [N]                 top kernels of a --stats kernel_stats.csv
    python tools/kstats.py --split TRACE_CSV STEPS [N]   the same from a --kernel-trace kernel_trace.csv, split into
                                                        the timed steps' kernels and setup/parity kernels (needs a
                                                        bench.py run with QVIT_STEP_MARKERS=1: its two spin kernels
                                                        bracket the timed steps)
    python tools/kstats.py --pmc FETCH_DIR WRITE_DIR [--round r01]
                                                        fc1 HBM traffic per launch from two PMC passes

PMC conventions (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are kilobytes per
dispatch; on gfx950 FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read (128-B requests
tallied at 64 B), so it is doubled; WRITE_SIZE is taken as is. Both count Infinity-Cache hits as
fabric traffic (an upper bound on HBM bytes).
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

FC1_KERNEL = re.compile(r"gemm_kernel<4, 2, 1(, (true|false|\d))?(, (true|false))?>")  # W4 weights, I8_GELU epilogue, 4 waves (any weight image, ring)


def top(path, n=25):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:n]:
        name = r["Name"]
        m = re.match(r"(?:void )?(?:\(anonymous namespace\)::)?([\w:<>, ]+?)\(", name)
        short = (m.group(1) if m else name)[:70]
        if short.startswith("Cijk"):
            short = name[:40]
        print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms  calls={int(r["Calls"]):5d}  '
              f'avg={float(r["AverageNs"])/1e3:9.2f} us  {float(r["Percentage"]):5.1f}%  {short}')


def _short(name):
    m = re.match(r"(?:void )?(?:\(anonymous namespace\)::)?([\w:<>, ]+?)\(", name)
    short = (m.group(1) if m else name)[:70]
    return name[:40] if short.startswith("Cijk") else short


def _table(rows, total, n, per=1):
    out = []
    for name, (calls, ns) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:n]:
        out.append(f"{ns / 1e6 / per:9.3f} ms  calls={calls / per:7.1f}  avg={ns / calls / 1e3:9.2f} us  "
                   f"{100.0 * ns / total if total else 0.0:5.1f}%  {_short(name)}")
    return out


def split(trace, steps, n=30):
    """Kernels dispatched between the two marker spin kernels of bench.py (QVIT_STEP_MARKERS=1) are the timed steps'
    kernels; everything before the first / after the second marker (library build checks, calibration, epilogue
    tables, the event-timed second pass, parity/reference launches) is setup/parity."""
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit(f"{trace}: {len(marks)} marker spin kernels (run bench.py with QVIT_STEP_MARKERS=1)")
    a, b = marks[0], marks[1]
    step, other = {}, {}
    for i, r in enumerate(rows):
        if i in (a, b):
            continue
        d = step if a < i < b else other
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        c = d.setdefault(r["Kernel_Name"], [0, 0])
        c[0] += 1
        c[1] += ns
    span = int(rows[b]["Start_Timestamp"]) - int(rows[a]["End_Timestamp"])
    st = sum(v[1] for v in step.values())
    ot = sum(v[1] for v in other.values())
    lines = [f"== timed steps: {steps} steps, {sum(v[0] for v in step.values())} dispatches "
             f"({sum(v[0] for v in step.values()) / steps:.1f} per step), kernel time {st / 1e6 / steps:.3f} ms per step, "
             f"marker-to-marker span {span / 1e6 / steps:.3f} ms per step (rows: per step)"]
    lines += _table(step, st, n, per=steps)
    lines += ["", f"== setup / calibration / event-timed pass / parity (NOT the step): "
                  f"{sum(v[0] for v in other.values())} dispatches, {ot / 1e6:.3f} ms total (rows: whole run)"]
    lines += _table(other, ot, n)
    print("\n".join(lines))


def pmc_values(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and FC1_KERNEL.search(r.get("Kernel_Name", "")):
                vals.append(float(r["Counter_Value"]))
    return vals


def _build_id():
    """The profiled library's build id, as quantized_vit_amd._lib.build_id computes it (the digest of its build
    inputs that build.py writes beside it; the bytes' sha256 without one) — no torch import needed."""
    import hashlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "quantized_vit_amd", "libqvit_hip.so")
    try:
        with open(lib + ".srcsha") as f:
            digest = f.read().strip()
        if digest:
            return "src-" + digest[:16]
    except OSError:
        pass
    try:
        with open(lib, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def pmc(fetch_dir, write_dir, rnd):
    fetch = pmc_values(fetch_dir, "FETCH_SIZE")
    write = pmc_values(write_dir, "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit(f"fc1 kernel not found in PMC output (fetch {len(fetch)}, write {len(write)})")
    f_b = 2.0 * statistics.median(fetch) * 1024
    w_b = statistics.median(write) * 1024
    out = {
        "kernel": FC1_KERNEL.pattern,
        "launches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "fetch_size_kb_median_raw": statistics.median(fetch),
        "write_size_kb_median_raw": statistics.median(write),
        "fetch_bytes_per_launch": f_b,
        "write_bytes_per_launch": w_b,
        "traffic_bytes_per_launch": f_b + w_b,
        "corrections": "FETCH_SIZE x2 (gfx950 64-B tally of 128-B requests), KB->B x1024; WRITE_SIZE as is",
        "round": rnd,
        "lib_build_id": _build_id(),
        # the profiled command: bench.py defaults (tools/profile_fc1.sh)
        "batch": int(os.environ.get("BENCH_BATCH", "256")),
        "model": os.environ.get("BENCH_MODEL", "vit_base_patch16_224"),
    }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    dirs = [os.path.join(root, "profiles")]
    if os.environ.get("PMC_OUT"):   # on the GPU box only gpurun_out/ travels back
        dirs.append(os.environ["PMC_OUT"])
    for d in dirs:
        os.makedirs(d, exist_ok=True)
        for name in (f"fc1_traffic_{rnd}.json", "fc1_traffic.json"):
            with open(os.path.join(d, name), "w") as fh:
                json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--pmc":
        rnd = sys.argv[sys.argv.index("--round") + 1] if "--round" in sys.argv else "r01"
        pmc(sys.argv[2], sys.argv[3], rnd)
    elif sys.argv[1] == "--split":
        split(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 30)
    else:
        top(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)

"""Median PMC counters of one kernel (name regex) over rocprofv3 --pmc pass directories, with the derived
fractions of MI355X_MICROARCH.md (GRBM_GUI_ACTIVE summed over 8 XCDs; MFMA busy over CUs x 4 SIMDs; SQ_*
wave counters in quad-cycles).   python tools/pmc_kernel.py 'ultra_conv0_mfma' DIR [DIR ...]"""
import csv
import glob
import os
import re
import statistics
import sys

CUS = 256


def main():
    pat = re.compile(sys.argv[1])
    vals, durs = {}, []
    for d in sys.argv[2:]:
        trace = {}
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if pat.search(r["Kernel_Name"]):
                    trace[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        durs += list(trace.values())
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if pat.search(r["Kernel_Name"]):
                    vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    med = {k: statistics.median(v) for k, v in vals.items()}
    dur = statistics.median(durs) if durs else 0.0
    print(f"dispatches {len(durs)}  median duration {dur / 1e3:.1f} us")
    for k in sorted(med):
        print(f"  {k:28s} {med[k]:.4g}")
    g = med.get("GRBM_GUI_ACTIVE")
    if g and dur:
        cyc = g / 8
        print(f"  clock {cyc / dur:.3f} GHz")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
            print(f"  MFMA busy {med['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * CUS * 4):.3f}")
        if "SQ_WAVE_CYCLES" in med:
            w = med["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if k in med:
                    print(f"  {k} / SQ_WAVE_CYCLES {med[k] / w:.3f}")
    if "FETCH_SIZE" in med:
        print(f"  HBM fetch {2 * med['FETCH_SIZE'] * 1024 / 1e6:.1f} MB (x2 gfx950)")
    if "SQ_LDS_BANK_CONFLICT" in med and "SQ_LDS_IDX_ACTIVE" in med:
        print(f"  LDS conflict share {med['SQ_LDS_BANK_CONFLICT'] / max(med['SQ_LDS_IDX_ACTIVE'], 1):.3f}")


if __name__ == "__main__":
    main()

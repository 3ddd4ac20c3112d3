"""Per-kernel medians of every PMC counter found under a tools/profile_pmc.sh output directory, plus the
derived ratios used in DESIGN.md (average VMEM / L2 latency, MFMA busy, wait fractions)."""
import collections
import csv
import glob
import os
import re
import statistics
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(\w+<[^>]*>|\w+)\(", r.get("Kernel_Name", ""))
        k = m.group(1) if m else r.get("Kernel_Name", "")[:60]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    med = {c: statistics.median(v) for c, v in cs.items()}
    print(f"== {k}")
    for c in sorted(med):
        print(f"   {c:34s} {med[c]:16.0f}")
    g = lambda c: med.get(c)
    der = []
    if g("SQ_INST_LEVEL_VMEM") and g("SQ_INSTS_VMEM"):
        der.append(f"avg VMEM latency (quad-cycles x4?) {g('SQ_INST_LEVEL_VMEM') / g('SQ_INSTS_VMEM'):.0f}")
    if g("TCP_TCC_READ_REQ_LATENCY") and g("TCP_TCC_READ_REQ"):
        der.append(f"avg L1->L2 read latency {g('TCP_TCC_READ_REQ_LATENCY') / g('TCP_TCC_READ_REQ'):.0f} cyc")
    if g("TCC_HIT") and g("TCC_MISS") is not None:
        der.append(f"L2 hit {100 * g('TCC_HIT') / (g('TCC_HIT') + g('TCC_MISS')):.1f}%")
    if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
        der.append(f"MFMA busy/(GUI_ACTIVE*CUs) {g('SQ_VALU_MFMA_BUSY_CYCLES') / (g('GRBM_GUI_ACTIVE') / 8 * 256 * 4):.3f}")
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if g(c) and g("SQ_WAVE_CYCLES"):
            der.append(f"{c}/WAVE_CYCLES {g(c) / g('SQ_WAVE_CYCLES'):.2f}")
    if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_LDS_IDX_ACTIVE"):
        der.append(f"LDS conflict share {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.2f}")
    for x in der:
        print("   -> " + x)

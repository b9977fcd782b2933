"""Summarise tools/pmc_sq.sh output for one kernel: instruction mix per wave and the share of
wave time spent issuing, waiting on dependencies / issue, and waiting on s_waitcnt.
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md)."""
import collections, csv, glob, sys

d, kern = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "k_blend")
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(d + "/p*/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
res = {c: sum(v.values()) / len(v) for c, v in agg.items()}
w = res["SQ_WAVES"]
cyc = res["GRBM_GUI_ACTIVE"] / 8  # summed over 8 XCDs
print(f"{d} [{kern}] kernel ~{cyc / 2.4e3:.1f} us at 2.4 GHz, {w:.0f} waves")
print(f"  per wave: VALU {res['SQ_INSTS_VALU'] / w:.0f}  SALU {res['SQ_INSTS_SALU'] / w:.0f}  "
      f"LDS {res['SQ_INSTS_LDS'] / w:.0f}  VMEM_RD {res['SQ_INSTS_VMEM_RD'] / w:.1f}")
wc = res["SQ_WAVE_CYCLES"]
print(f"  wave time: issuing {res['SQ_ACTIVE_INST_ANY'] / wc:.0%}  wait-inst {res['SQ_WAIT_INST_ANY'] / wc:.0%}  "
      f"waitcnt {res['SQ_WAIT_ANY'] / wc:.0%}; resident waves/SIMD {4 * wc / cyc / 1024:.1f}")
print(f"  VALU pipe busy (2 cyc/instr) {res['SQ_INSTS_VALU'] * 2 / 1024 / cyc:.0%}")

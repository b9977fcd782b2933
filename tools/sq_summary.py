"""Summarise tools/pmc_sq.sh output for one kernel: instruction mix per wave and the share of
wave time spent issuing, waiting on dependencies / issue, and waiting on s_waitcnt.
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md);
GRBM_GUI_ACTIVE is summed over the 8 XCDs.

Usage: python tools/sq_summary.py gpurun_out/prof_<tag>_<config> [kernel-substring] [--json out.json]
--json writes the per-launch averages of every counter (keyed by the kernel substring) and the
profiled library's sha (lib.sha, tools/profile_config.sh), which bench.py matches against the
library it loads for the blend's VALU roofline."""
import collections
import csv
import glob
import json
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
d, kern = args[0], (args[1] if len(args) > 1 else "k_blend")
out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
if out_json in args:
    args.remove(out_json)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
names = set()
for f in glob.glob(d + "/p[0-9]*/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            names.add(r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0])
            agg[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
res = {c: sum(v.values()) / len(v) for c, v in agg.items()}
launches = {c: len(v) for c, v in agg.items()}
w = res["SQ_WAVES"]
cyc = res["GRBM_GUI_ACTIVE"] / 8  # summed over 8 XCDs
print(f"{d} [{kern}] kernel ~{cyc / 2.4e3:.1f} us at 2.4 GHz, {w:.0f} waves")
print(f"  per wave: VALU {res['SQ_INSTS_VALU'] / w:.0f}  SALU {res['SQ_INSTS_SALU'] / w:.0f}  "
      f"LDS {res['SQ_INSTS_LDS'] / w:.0f}  VMEM_RD {res['SQ_INSTS_VMEM_RD'] / w:.1f}")
print(f"  per launch: VALU {res['SQ_INSTS_VALU'] / 1e6:.1f} M wave-instructions")
if "SQ_WAVE_CYCLES" in res and "SQ_ACTIVE_INST_ANY" in res:
    wc = res["SQ_WAVE_CYCLES"]
    print(f"  wave time: issuing {res['SQ_ACTIVE_INST_ANY'] / wc:.0%}  "
          f"wait-inst {res['SQ_WAIT_INST_ANY'] / wc:.0%}  waitcnt {res['SQ_WAIT_ANY'] / wc:.0%}; "
          f"resident waves/SIMD {4 * wc / cyc / 1024:.1f}")
print(f"  VALU pipe busy (2 cyc/instr) {res['SQ_INSTS_VALU'] * 2 / 1024 / cyc:.0%}")
if "SQ_ACTIVE_INST_VALU" in res:
    # counts instructions, like SQ_INSTS_VALU (tools/micro/valu_calib.hip: both read exactly
    # the known count of a calibration kernel; profiles/r02_valu_calibration.md)
    print(f"  SQ_ACTIVE_INST_VALU {res['SQ_ACTIVE_INST_VALU'] / 1e6:.1f} M (= VALU instructions)")
if out_json:
    import os
    sha = os.path.join(d, "lib.sha")
    json.dump({"kernel": kern, "kernels_matched": sorted(names), "source": d,
               "lib_sha16": open(sha).read().strip() if os.path.exists(sha) else None,
               "launches": launches, "per_launch": res}, open(out_json, "w"), indent=1)
    print("wrote", out_json)

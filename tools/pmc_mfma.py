#!/usr/bin/env python3
"""Per-kernel MFMA-busy and wave-stall counters from one rocprofv3 PMC pass
(MI355X_MICROARCH.md "rocprofv3 PMC slots": 8 SQ + 2 GRBM counters fit one pass):

  SQ_VALU_MFMA_BUSY_CYCLES  SIMD-cycles an MFMA occupied (32 per v_mfma_f32_32x32x16_f16)
  GRBM_GUI_ACTIVE           GPU-busy cycles, summed over the 8 XCDs
  SQ_WAVE_CYCLES            wave-cycles (quad-cycles), = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
  SQ_WAIT_ANY               waves parked at s_waitcnt / barriers
  SQ_WAIT_INST_ANY          issue stalls (MFMA dependency, pipe busy)
  SQ_ACTIVE_INST_ANY        cycles issuing
  SQ_WAIT_INST_LDS          LDS-issue stalls (a part of WAIT_INST_ANY)
  SQ_INSTS_LDS              LDS instructions issued

Derived per launch, keyed by the profiler sections of tools/pmc_traffic.py:
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of
      the chip's SIMD-cycles (over the kernel's busy time) spent in MFMAs;
  wait_any / wait_inst / active = their share of SQ_WAVE_CYCLES.
Usage: tools/pmc_mfma.py <workload> <pmc_dir> <out.json>
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_traffic as P  # noqa: E402

COUNTERS = ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
            "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_INSTS_LDS",
            "SQ_BUSY_CYCLES"]


def main():
    workload, d, out = sys.argv[1:4]
    P.TABLE = P.TABLES[workload]
    paths = sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True),
                   key=os.path.getmtime)[-1:]
    # (section, dispatch) -> counter -> value (a counter may be reported per dimension:
    # summed per dispatch)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in paths:
        for r in csv.DictReader(open(path)):
            sec = P.section(r["Kernel_Name"], r.get("Grid_Size"))
            if sec:
                per[(sec, r.get("Dispatch_Id") or r.get("Correlation_Id"))][r["Counter_Name"]] += \
                    float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (sec, _), c in per.items():
        for k, v in c.items():
            agg[sec][k].append(v)
    res = {}
    for sec, c in agg.items():
        m = {k: sum(v) / len(v) for k, v in c.items()}
        row = {k: round(v) for k, v in m.items()}
        g = m.get("GRBM_GUI_ACTIVE", 0.0)
        if g > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            row["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * g / 8.0), 4)
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        if wc > 0:
            for k, name in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst"),
                            ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_WAIT_INST_LDS", "wait_lds")):
                if k in m:
                    row[name] = round(m[k] / wc, 4)
        row["launches"] = len(next(iter(c.values())))
        res[sec] = row
    names = sorted({k for c in agg.values() for k in c})
    json.dump({"method": "rocprofv3 --pmc " + " ".join(names) + " (one pass, kernels "
               "serialised by the counter collection); mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / "
               "(1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); wait_* / active = share of "
               "SQ_WAVE_CYCLES; per launch", "kernels": res}, open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in v:
            print(f"{k:22s} " + " ".join(f"{n}={v[n]}" for n in names if n in v))
            continue
        print(f"{k:22s} mfma_busy {v.get('mfma_busy', float('nan')):.3f}  wait_any "
              f"{v.get('wait_any', float('nan')):.3f}  wait_inst {v.get('wait_inst', float('nan')):.3f}"
              f"  active {v.get('active', float('nan')):.3f}  wait_lds {v.get('wait_lds', float('nan')):.3f}")


if __name__ == "__main__":
    main()

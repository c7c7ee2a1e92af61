"""Per-kernel SQ (shader sequencer) counters from rocprofv3 --pmc passes of a bench run:
    python tools/sq_summary.py OUT.json PASS_DIR [PASS_DIR ...]
Averages every SQ_* counter per dispatch of each kernel symbol and derives
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES / 32 * 1024)
i.e. the fraction of SIMD-cycles the matrix pipe was busy while the kernel ran: MFMA busy cycles
are per SIMD (= 16 per v_mfma_f32_16x16x32_bf16, MI355X_MICROARCH.md constants table), the 1,024
SIMDs are 256 CUs x 4, and SQ_BUSY_CYCLES sums the busy cycles of the 32 shader engines' SQs
(checked: the fused MLP's SQ_BUSY_CYCLES / 32 equals its launch duration x clock).
  wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES  (share of wave lifetime spent waiting, any reason)
  lds_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (conflict cycles per LDS instruction)
bench.py's roofline reads mfma_busy of the dominant kernel from profiles/*_<cfg>_sq.json."""
import collections
import csv
import glob
import json
import sys


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in sorted(acc.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        row = {"dispatches": max(len(v) for v in cs.values()), **{c: round(v) for c, v in sorted(avg.items())}}
        if avg.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            row["mfma_busy"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["SQ_BUSY_CYCLES"] / 32 * 1024), 4)
        if avg.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in avg:
            row["wait_frac"] = round(avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"], 4)
        if avg.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in avg:
            row["lds_conflict_per_inst"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_INSTS_LDS"], 3)
        out[k] = row
    json.dump(out, open(out_path, "w"), indent=1)
    for k, v in out.items():
        if "mfma_busy" in v and v["SQ_VALU_MFMA_BUSY_CYCLES"] > 1e6:
            print(f"{k[:70]:70s} mfma_busy {v['mfma_busy']:.3f} wait {v.get('wait_frac', 0):.2f}")


if __name__ == "__main__":
    main()

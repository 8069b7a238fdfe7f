"""Per-kernel-dispatch PMC summary of rocprofv3 counter CSVs (one or more passes): averages per
kernel name; MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * CUs) style ratios."""
import collections
import csv
import glob
import sys


def main():
    root = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            agg[name]["_dur_us"].append(dur)
    for name, c in agg.items():
        if "conv" not in name and "gemm" not in name:
            continue
        avg = {k: sum(v) / len(v) for k, v in c.items()}
        line = {k: round(v, 1) for k, v in avg.items()}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "SQ_BUSY_CYCLES" in avg and avg["SQ_BUSY_CYCLES"]:
            line["mfma_busy_per_busy"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / avg["SQ_BUSY_CYCLES"], 3)
        print(name, line)


if __name__ == "__main__":
    main()

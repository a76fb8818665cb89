"""Per-dispatch memory counters of the verify kernels from rocprofv3 --pmc
passes (one counter group per pass; tools/gpu_measure.sh): FETCH_SIZE and
WRITE_SIZE (KiB), TCC_HIT_sum / TCC_MISS_sum (L2 requests). Counter rows of
one dispatch (one per instance) are summed, then averaged over the
kernel's dispatches of each grid size.

    python tools/l2_traffic.py <out.json> <pass_dir> [<pass_dir> ...]
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> sum
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                key = f"{name} grid={int(r['Grid_Size']) // 64} waves"
                acc[key][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    doc = {}
    for k, cs in acc.items():
        doc[k] = {c: {"mean_per_dispatch": sum(v.values()) / len(v), "dispatches": len(v)} for c, v in cs.items()}
        e = doc[k]
        if "FETCH_SIZE" in e:
            e["fetch_bytes_raw"] = e["FETCH_SIZE"]["mean_per_dispatch"] * 1024
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e:
            h, m = e["TCC_HIT_sum"]["mean_per_dispatch"], e["TCC_MISS_sum"]["mean_per_dispatch"]
            e["l2_hit_rate"] = h / (h + m) if h + m else None
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k in sorted(doc):
        print(k, json.dumps({c: round(v["mean_per_dispatch"], 1) if isinstance(v, dict) else v
                             for c, v in doc[k].items()}))


if __name__ == "__main__":
    main()

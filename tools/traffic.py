"""Per-launch HBM traffic of the bench's verify kernel from rocprofv3 PMC
passes (one counter group per pass). FETCH_SIZE / WRITE_SIZE are in KiB.
bytes_per_launch is the RAW figure (what bench.py reports): the guide's x2
FETCH_SIZE correction for gfx950 (/opt/skills/guides/MI355X_MICROARCH.md,
"HBM [CDNA4]") is calibrated on 16-B/lane streaming reads, and this kernel's
8-16 B per-lane row loads match the algorithmic bytes without it (DESIGN.md
5); the corrected figure is kept beside it.

    python tools/traffic.py <pmc_fetch_dir> <pmc_write_dir> <out.json> [kernel-substring]
"""
import csv
import glob
import json
import sys


def per_launch(d, counter, kname):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kname} in {f}")
    return sum(vals.values()) / len(vals), len(vals)


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    kname = sys.argv[4] if len(sys.argv) > 4 else "k_verify_quad"
    fk, nf = per_launch(fetch_dir, "FETCH_SIZE", kname)
    wk, nw = per_launch(write_dir, "WRITE_SIZE", kname)
    doc = {"kernel": kname, "dispatches": [nf, nw], "fetch_size_kib_raw": round(fk, 3),
           "write_size_kib_raw": round(wk, 3),
           "bytes_per_launch": round(fk * 1024 + wk * 1024),
           "bytes_per_launch_guide_corrected": round(2 * fk * 1024 + wk * 1024),
           "correction": "raw KiB -> bytes; guide-corrected = FETCH_SIZE x2 (wide-read calibration)"}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()

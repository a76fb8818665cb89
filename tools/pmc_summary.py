"""Summarize rocprofv3 --pmc counter CSVs per kernel (mean per dispatch).

  python tools/pmc_summary.py <out.txt> <pass_dir> [<pass_dir> ...]

Each pass dir holds run_counter_collection.csv from one `rocprofv3 --pmc`
run (tools/gpu_prof.sh).  For every kernel: dispatches, the mean value of
each counter per dispatch, and for the verify kernels the derived per-wave
figures (VALU instructions per wave, wave cycles per wave, VALU issue share
of wave time, wait share).
"""
import csv
import json
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(list))
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            key = f"{name} grid={int(r['Grid_Size']) // 64} waves"
            per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    merged = defaultdict(dict)
    disp = {}
    for d in dirs:
        for k, cs in load(d).items():
            for c, vals in cs.items():
                merged[k][c] = sum(vals) / len(vals)
                disp[k] = max(disp.get(k, 0), len(vals))
    lines = [f"# rocprofv3 --pmc, mean per dispatch; passes: {', '.join(os.path.basename(d) for d in dirs)}"]
    for k in sorted(merged, key=lambda k: -merged[k].get("SQ_INSTS_VALU", 0) * max(disp[k], 1)):
        cs = merged[k]
        lines.append(f"\n[{k}]  dispatches={disp[k]}")
        for c in sorted(cs):
            lines.append(f"  {c:24s} {cs[c]:18,.0f}")
        w = cs.get("SQ_WAVES")
        if w and "SQ_INSTS_VALU" in cs:
            lines.append(f"  -> VALU instructions / wave  {cs['SQ_INSTS_VALU'] / w:12,.0f}")
        if w and "SQ_WAVE_CYCLES" in cs:
            # SQ_WAVE_CYCLES counts in quad-cycles (4 clocks) on gfx950
            lines.append(f"  -> wave cycles / wave (x4)   {4 * cs['SQ_WAVE_CYCLES'] / w:12,.0f}")
            if "SQ_ACTIVE_INST_VALU" in cs:
                lines.append(f"  -> VALU-active share of wave {cs['SQ_ACTIVE_INST_VALU'] / cs['SQ_WAVE_CYCLES']:12.3f}")
            if "SQ_WAIT_ANY" in cs:
                lines.append(f"  -> waiting share of wave     {cs['SQ_WAIT_ANY'] / cs['SQ_WAVE_CYCLES']:12.3f}")
        if "SQ_ACTIVE_INST_VALU" in cs and cs.get("GRBM_GUI_ACTIVE"):
            # VALUBusy (chip-wide): active VALU quad-cycles x 4 over SIMDs x
            # per-XCD GPU-busy cycles (GRBM_GUI_ACTIVE sums the 8 XCDs)
            busy = 100 * cs["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (cs["GRBM_GUI_ACTIVE"] / 8)
            lines.append(f"  -> VALUBusy (chip, %)        {busy:12.1f}")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    # the derived figures as JSON beside the text (bench.py reads VALUBusy)
    derived = {}
    for k, cs in merged.items():
        w = cs.get("SQ_WAVES")
        dd = {"dispatches": disp[k]}
        if w and "SQ_INSTS_VALU" in cs:
            dd["valu_insts_per_wave"] = round(cs["SQ_INSTS_VALU"] / w)
        if w and "SQ_WAVE_CYCLES" in cs:
            dd["wave_cycles_per_wave"] = round(4 * cs["SQ_WAVE_CYCLES"] / w)
        if "SQ_ACTIVE_INST_VALU" in cs and cs.get("GRBM_GUI_ACTIVE"):
            dd["valu_busy_pct"] = round(100 * cs["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (cs["GRBM_GUI_ACTIVE"] / 8), 1)
        derived[k] = dd
    with open(os.path.splitext(out)[0] + ".json", "w") as f:
        json.dump(derived, f, indent=1)
    print("\n".join(lines[:60]))


if __name__ == "__main__":
    main()

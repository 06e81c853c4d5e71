"""Reduce rocprofv3 --pmc counter CSVs (scripts/archive/gpu_narrow_pmc.sh passes) to one JSON:
per kernel instance, the mean of each counter over its dispatches, plus derived ratios
(wait / active shares of wave cycles, VALU and LDS instructions per MFMA, MFMA busy share).

    python tools/sq_summary.py gpurun_out TAG > TAG_summary.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root, tag = sys.argv[1], sys.argv[2]
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(set))
    for d in sorted(glob.glob(os.path.join(root, f"{tag}_s*_p*"))):
        if not os.path.isdir(d):
            continue
        shape = os.path.basename(d).split("_")[-2]
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = f"{shape} {r['Kernel_Name'].replace('void ', '').split('(')[0]}"
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[k][r["Counter_Name"]].add(r["Dispatch_Id"])
    out = {}
    for k, d in acc.items():
        m = {c: v / max(len(cnt[k][c]), 1) for c, v in d.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        der = {}
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"):
                if c in m:
                    der[c + "/WAVE_CYCLES"] = round(m[c] / wc, 3)
        mf = m.get("SQ_INSTS_MFMA", 0.0)
        if mf:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD"):
                if c in m:
                    der[c + "/MFMA"] = round(m[c] / mf, 3)
        if m.get("SQ_WAVES"):
            der["wave_cycles_per_wave"] = round(wc / m["SQ_WAVES"], 1)
            if mf:
                der["mfma_per_wave"] = round(mf / m["SQ_WAVES"], 1)
        out[k] = {"counters": {c: round(v, 1) for c, v in sorted(m.items())}, "derived": der}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()

"""Per-launch HBM traffic of one kernel from rocprofv3 PMC passes.

    python tools/pmc_traffic.py --fetch DIR_FETCH --write DIR_WRITE \
        --kernel "igemm_kernel<4, 4, true, 0>" --out profiles/r1_pmc_traffic.json

Counters (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are in KiB and come
from separate passes.  On gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced read, so it is doubled for kernels whose loads are
16-byte buffer loads (the igemm kernels); WRITE_SIZE is exact for 16-B stores
and uncalibrated for the 4-B stores these kernels issue (noted in the output).
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics


def rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = []
    for f in files:
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def norm(name):
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("vae2::", "").replace("void ", "").strip()


def per_launch(d, counter, kernel):
    vals = {}
    for r in rows(d):
        if r.get("Counter_Name") != counter:
            continue
        if norm(r.get("Kernel_Name", "")) != kernel:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--fetch-scale", type=float, default=2.0)
    a = ap.parse_args()
    f = per_launch(a.fetch, "FETCH_SIZE", a.kernel)
    w = per_launch(a.write, "WRITE_SIZE", a.kernel)
    if not f or not w:
        raise SystemExit(f"no samples for {a.kernel}: fetch {len(f)} write {len(w)}")
    fetch_b = statistics.mean(f) * 1024 * a.fetch_scale
    write_b = statistics.mean(w) * 1024
    res = {"kernel": a.kernel, "launches_fetch": len(f), "launches_write": len(w),
           "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": fetch_b + write_b,
           "note": f"FETCH_SIZE x{a.fetch_scale} (gfx950 wide-read calibration), WRITE_SIZE x1 "
                   "(4-byte stores: uncalibrated width); KiB -> bytes x1024; mean over launches"}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""Per-step kernel-time breakdown from a rocprofv3 kernel trace (CSV).

    python vae-2_amd/tools/trace_steps.py gpurun_out/prof/run_kernel_trace.csv [--steps 10]

Steps are delimited by the Adam launches (the last kernel family of a step).
Reports, over the last --steps steps: wall span, GPU busy time (union of
kernel intervals across streams), summed kernel time by family, and the idle gap.
"""
import argparse
import csv
import re
from collections import defaultdict


def family(name):
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(.*$", "", n)
    if n.startswith("vae2::"):
        n = n[6:]
    if "igemm_kernel" in n:
        m = re.search(r"<(\d+), (\d+), (\w+), (\d+)>", n)
        role = {"0": "conv_fwd", "1": "conv_dgrad", "2": "conv_dgrad_s2"}.get(m.group(4), "igemm")
        return role
    n = re.sub(r"<.*", "", n)
    if "elementwise" in n or n.startswith("at::"):
        return "torch:" + n.split("::")[-1][:40]
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="adam")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    # group consecutive marker launches of one step (several flats)
    ends = []
    for i in marks:
        if ends and i - ends[-1] <= 4:
            ends[-1] = i
        else:
            ends.append(i)
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} steps found")
    lo, hi = ends[-a.steps - 1] + 1, ends[-1] + 1
    sel = rows[lo:hi]
    t0, t1 = sel[0][0], max(r[1] for r in sel)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    fam = defaultdict(lambda: [0, 0])
    for s, e, n in sel:
        f = family(n)
        fam[f][0] += e - s
        fam[f][1] += 1
    k = a.steps
    total = sum(v[0] for v in fam.values())
    print(f"steps {k}: wall/step {(t1 - t0) / k / 1e6:.2f} ms, busy/step {busy / k / 1e6:.2f} ms, "
          f"summed kernel/step {total / k / 1e6:.2f} ms, launches/step {len(sel) / k:.0f}")
    for f, (t, c) in sorted(fam.items(), key=lambda x: -x[1][0]):
        print(f"  {f:40s} {t / k / 1e6:8.2f} ms  {c / k:7.0f} launches  {t / c / 1e3:8.1f} us avg")


if __name__ == "__main__":
    main()

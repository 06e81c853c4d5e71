"""Per-step kernel-time breakdown from a rocprofv3 kernel trace (CSV).

    python vae-2_amd/tools/trace_steps.py gpurun_out/prof/run_kernel_trace.csv [--steps 10]
        [--instances N] [--json out.json]

Steps are delimited by the Adam launches (the last kernel family of a step).
Reports, over the last --steps steps: wall span, GPU busy time (union of
kernel intervals across streams), summed kernel time per family (conv fwd /
dgrad, weight-grad, BatchNorm, heads, fuse/resample, ...), per kernel, and the
top --instances kernel instantiations by time.
"""
import argparse
import csv
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from vae2.prof import family  # noqa: E402  (the families bench.py reports live)


def kernel_name(name):
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(.*$", "", n)
    return n[6:] if n.startswith("vae2::") else n


def short(n):
    """Kernel without template arguments (aten kernels shortened)."""
    if "at::native" in n:
        m = re.search(r"CUDAFunctor_(\w+)|(\w+Functor)|(direct_copy)", n)
        return "torch:" + (next(g for g in m.groups() if g) if m else n[:40])
    return re.sub(r"<.*", "", n)


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         kernel_name(r["Kernel_Name"]), int(r.get("Queue_Id") or 0)))
    rows.sort()
    return rows


def select_steps(rows, steps, marker="adam", skip=0):
    marks = [i for i, r in enumerate(rows) if marker in r[2]]
    ends = []  # group consecutive marker launches of one step (several flats)
    for i in marks:
        if ends and i - ends[-1] <= 4:
            ends[-1] = i
        else:
            ends.append(i)
    if skip:
        ends = ends[:-skip]
    if len(ends) < steps + 1:
        raise SystemExit(f"only {len(ends)} steps found")
    return rows[ends[-steps - 1] + 1:ends[-1] + 1]


def busy_ns(sel):
    busy, cur_s, cur_e = 0, None, None
    for s, e, *_ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return busy + (cur_e - cur_s)


def breakdown(sel, k):
    fam, ker, inst = (defaultdict(lambda: [0, 0]) for _ in range(3))
    for s, e, n, *_ in sel:
        for d, key in ((fam, family(n)), (ker, short(n)), (inst, n)):
            d[key][0] += e - s
            d[key][1] += 1
    t0, t1 = sel[0][0], max(r[1] for r in sel)
    total = sum(v[0] for v in fam.values())

    def table(d):
        return [{"name": n, "ms_per_step": t / k / 1e6, "launches_per_step": c / k,
                 "avg_us": t / c / 1e3} for n, (t, c) in sorted(d.items(), key=lambda x: -x[1][0])]

    queues = defaultdict(list)
    for r in sel:
        queues[r[3] if len(r) > 3 else 0].append(r)
    qt = [{"queue": q, "busy_ms_per_step": busy_ns(v) / k / 1e6,
           "kernel_ms_per_step": sum(e - s for s, e, *_ in v) / k / 1e6,
           "launches_per_step": len(v) / k} for q, v in sorted(queues.items())]
    return {"steps": k, "wall_ms_per_step": (t1 - t0) / k / 1e6, "queues": qt,
            "busy_ms_per_step": busy_ns(sel) / k / 1e6, "kernel_ms_per_step": total / k / 1e6,
            "launches_per_step": len(sel) / k, "families": table(fam), "kernels": table(ker),
            "instances": table(inst)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="adam")
    ap.add_argument("--instances", type=int, default=25)
    ap.add_argument("--skip", type=int, default=0,
                    help="leave out the last N steps (bench.py's eager roofline steps: the "
                         "graph-replayed timed steps come before them)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    b = breakdown(select_steps(load(a.csv), a.steps, a.marker, a.skip), a.steps)
    print(f"steps {b['steps']}: wall/step {b['wall_ms_per_step']:.2f} ms, busy/step "
          f"{b['busy_ms_per_step']:.2f} ms, summed kernel/step {b['kernel_ms_per_step']:.2f} ms, "
          f"launches/step {b['launches_per_step']:.0f}")
    print("-- hardware queues (HIP streams): busy = union of the queue's kernel intervals")
    for q in b["queues"]:
        print(f"  queue {q['queue']:3d}  busy {q['busy_ms_per_step']:7.2f} ms  kernels "
              f"{q['kernel_ms_per_step']:7.2f} ms  {q['launches_per_step']:7.1f} launches")
    for title, key, lim in (("families", "families", None), ("kernels", "kernels", None),
                            ("top instances", "instances", a.instances)):
        print(f"-- {title}")
        for r in b[key][:lim]:
            print(f"  {r['name'][:60]:60s} {r['ms_per_step']:8.2f} ms  "
                  f"{r['launches_per_step']:7.1f} launches  {r['avg_us']:8.1f} us avg")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(b, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""How much of each memory-bound kernel of the forward runs under a conv on the other stream.

Reads a rocprofv3 --kernel-trace CSV of `bench.py` (default --split 2: the forward runs as two part-batch
forwards on two streams, so the small kernels of one part -- InstanceNorm++ finalize, max-pools, the
head convs -- can run beside the other part's convs) and reports, per kernel class, the summed duration
and the part of it during which a conv_mfma_kernel dispatch of ANOTHER queue was executing (interval
intersection against the union of those conv intervals).  A class whose `hidden_frac` is ~1 costs the
step nothing beyond its share of the chip while it runs.

usage: tools/overlap.py <run_kernel_trace.csv> [out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict

CLASSES = [("inpp_moments", "inpp_moments_kernel"), ("inpp_ss", "inpp_ss_kernel"), ("maxpool5", "maxpool5_kernel"),
           ("avgpool2", "avgpool2_kernel"), ("begin_conv", "begin_conv"), ("end_conv+langevin", "end_conv"),
           ("merge", "merge_")]


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def covered(a, b, u):
    """length of [a, b) covered by the sorted disjoint intervals u"""
    s = 0
    for x, y in u:
        if y <= a:
            continue
        if x >= b:
            break
        s += min(b, y) - max(a, x)
    return s


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    conv = defaultdict(list)                     # queue -> conv intervals
    for r in rows:
        if "conv_mfma_kernel" in r["Kernel_Name"]:
            conv[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    queues = sorted(conv)
    other = {q: union([iv for q2 in queues if q2 != q for iv in conv[q2]]) for q in set(r["Queue_Id"] for r in rows)}
    agg = defaultdict(lambda: [0, 0, 0])         # class -> [dispatches, ns, hidden ns]
    for r in rows:
        n = r["Kernel_Name"]
        for cls, pat in CLASSES:
            if pat in n:
                a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                g = agg[cls]
                g[0] += 1
                g[1] += b - a
                g[2] += covered(a, b, other.get(r["Queue_Id"], []))
                break
    conv_ns = sum(b - a for q in queues for a, b in conv[q])
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                    "simultaneous-diffusion-for-pointclouds_amd"))
    from sdp import _build
    doc = {"trace": sys.argv[1], "libsdp_source_hash": _build.source_hash(), "queues_with_convs": len(queues),
           "conv_kernel_ns": conv_ns,
           "classes": {c: {"dispatches": v[0], "total_us": round(v[1] / 1e3, 1), "hidden_us": round(v[2] / 1e3, 1),
                           "hidden_frac": round(v[2] / v[1], 4) if v[1] else None} for c, v in sorted(agg.items())}}
    print(json.dumps(doc, indent=1))
    if len(sys.argv) > 2:
        json.dump(doc, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()

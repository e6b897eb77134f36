"""Average L2->EA read/write bytes per dispatch of a rocprofv3 --pmc run (gfx950 corrections:
reads x 128 B per TCC_EA0_RDREQ, writes 64/32 B per WRREQ_64B / other WRREQ)."""
import collections
import csv
import glob
import sys

d = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
rd = [v["TCC_EA0_RDREQ_sum"] * 128 for v in d.values()]
wr = [64 * v["TCC_EA0_WRREQ_64B_sum"] + 32 * (v["TCC_EA0_WRREQ_sum"] - v["TCC_EA0_WRREQ_64B_sum"]) for v in d.values()]
n = len(rd)
print(f"{sys.argv[1]}: {n} dispatches, read {sum(rd) / n / 1e6:.1f} MB, write {sum(wr) / n / 1e6:.1f} MB per launch")

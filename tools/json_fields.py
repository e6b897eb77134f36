"""Print selected (dotted) fields of a JSON line read from stdin."""
import json
import sys

d = json.loads(sys.stdin.read())
out = []
for f in sys.argv[1:]:
    v = d
    for k in f.split("."):
        v = v[k]
    out.append(str(v))
print(" ".join(out))

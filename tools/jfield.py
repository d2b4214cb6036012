"""Print selected fields of the JSON document on stdin: python tools/jfield.py us.infer us.infer_accumulate_fused"""
import json
import sys

doc = json.load(sys.stdin)
out = {}
for path in sys.argv[1:]:
    v = doc
    for k in path.split("."):
        v = v[k]
    out[path] = round(v, 2) if isinstance(v, float) else v
print(json.dumps(out))

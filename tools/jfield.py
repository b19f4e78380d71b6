#!/usr/bin/env python3
"""Print fields of a one-line JSON result: python tools/jfield.py FILE key [key ...]"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(" ".join(f"{k}={json.dumps(d.get(k))}" for k in sys.argv[2:]))

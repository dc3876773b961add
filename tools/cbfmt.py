"""Compact table of convbench JSON lines (stdin)."""
import json
import sys

for line in sys.stdin:
    if line.startswith("{"):
        d = json.loads(line)
        print(f"  {d['shape']:>14} {d['op']:>5} {d['kernel'][:34]:34} {d['us']:7.1f} us {d['tflops']:6.1f} TF")

"""Merge one bench.py DK_VERBOSE=1 DK_CONSUME_PROFILE=1 log into per-step timelines on one clock:
the open's [dk] events (relative to the 64-file open's start) and the consumer's batch arrivals.

    python tools/timeline_merge.py gpurun_out/<tag>/bench.err
"""
import ast
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
step, t0 = None, None
for ln in lines:
    m = re.match(r"\[dk\] open of (\d+) files starts at monotonic ([\d.]+) ms", ln)
    if m:
        if int(m.group(1)) > 1:
            t0 = float(m.group(2)); step = (step or 0) + 1
            print("==== step %d" % step)
        continue
    if t0 is None:
        continue
    if ln.startswith("[dk] "):
        print("   ", ln[5:])
    elif ln.startswith("consume starts"):
        m = re.match(r"consume starts at monotonic ([\d.]+) ms; arrivals \(monotonic ms, file, rows\): (\[.*\]) ; ends at monotonic ([\d.]+) ms", ln)
        if not m:
            print("?? unparsed consume line"); continue
        c0, arr, c1 = float(m.group(1)), ast.literal_eval(m.group(2)), float(m.group(3))
        print("    consume starts at %.1f ms" % (c0 - t0))
        prev = c0
        for t, f, n in arr:
            print("      batch file %3d (%d rows) at %.1f ms (+%.1f)" % (f, n, t - t0, t - prev)); prev = t
        print("    consume ends at %.1f ms" % (c1 - t0))

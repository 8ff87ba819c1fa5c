"""Copies the `_delta_log` of selected reference golden tables into tests/golden/tables/ (data
fixtures: inputs) and records the oracle's answers for them in tests/golden/expected.json (outputs).
The oracle itself is pinned to the answers the reference's tests assert
(tests/test_oracle_golden.py). Run in the container that has /root/reference:

    python tests/golden/make_fixtures.py
"""
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import ref  # noqa: E402

GOLD = "/root/reference/connectors/golden-tables/src/main/resources/golden"
KDRES = "/root/reference/kernel/kernel-defaults/src/test/resources"
TABLES = {
    "checkpoint": GOLD, "snapshot-data3": GOLD, "snapshot-repartitioned": GOLD, "log-replay-dv-key-cases": GOLD,
    "log-replay-special-characters-a": GOLD, "log-replay-special-characters-b": GOLD,
    "delete-re-add-same-file-different-transactions": GOLD, "multi-part-checkpoint": GOLD,
    "basic-with-inserts-deletes-checkpoint": GOLD, "only-checkpoint-files": GOLD, "v2-checkpoint-parquet": GOLD,
    "v2-checkpoint-json": GOLD,
    "dv-partitioned-with-checkpoint": GOLD, "data-skipping-basic-stats-all-types-checkpoint": GOLD,
    "data-skipping-basic-stats-all-types": GOLD, "data-skipping-basic-stats-all-types-columnmapping-name": GOLD,
    "data-skipping-basic-stats-all-types-columnmapping-id": GOLD,
    "data-skipping-change-stats-collected-across-versions": GOLD, "data-skipping-partition-and-data-column": GOLD,
    "basic-dv-with-checkpoint": KDRES, "basic-with-checkpoint": KDRES,
    "data-reader-partition-values": GOLD, "data-reader-timestamp_ntz": GOLD,
    "data-reader-timestamp_ntz-name-mode": GOLD, "data-reader-timestamp_ntz-id-mode": GOLD,
}


def canon_json(rows):
    """Rows as JSON; the machine-dependent tableRoot prefix becomes ${TABLES} (tests/golden_util.py)."""
    from tests.golden_util import to_json_rows
    return to_json_rows(rows)


def main():
    out = {}
    for name, base in TABLES.items():
        src = os.path.join(base, name, "_delta_log")
        if not os.path.isdir(src):
            print("skip", name)
            continue
        dst = os.path.join(HERE, "tables", name, "_delta_log")
        shutil.rmtree(os.path.dirname(dst), ignore_errors=True)
        shutil.copytree(src, dst, ignore=shutil.ignore_patterns("*.crc", ".*.crc"))
        res = {}
        for bs in (2, 1024):
            for stats in (False, True):
                r = ref.replay(os.path.dirname(dst), json_batch_size=bs, with_stats=stats)
                res["%d-%d" % (bs, int(stats))] = {"version": r.version, "counters": list(r.counters.as_tuple()),
                                                   "rows": canon_json(r.scan_files())}
        out[name] = res
        print(name, res["1024-0"]["version"], len(res["1024-0"]["rows"]), res["1024-0"]["counters"])
    with open(os.path.join(HERE, "expected.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()

import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
TABLES = os.path.join(HERE, "golden", "tables")


def load_expected():
    with open(os.path.join(HERE, "golden", "expected.json")) as f:
        return json.load(f)


def tables_uri():
    """The tableRoot prefix of the committed tables (machine dependent; fixtures store ${TABLES})."""
    from oracle import ref
    return ref.table_root_uri(TABLES)


def to_json_rows(rows):
    prefix = tables_uri()

    def enc(x):
        if isinstance(x, str) and x.startswith(prefix + "/"):
            return "${TABLES}" + x[len(prefix):]
        if isinstance(x, bytes):
            return {"b": x.decode("utf-8", "surrogateescape")}
        if isinstance(x, tuple):
            return [enc(v) for v in x]
        return x
    return [enc(r) for r in rows]

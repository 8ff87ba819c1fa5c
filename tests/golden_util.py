import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
TABLES = os.path.join(HERE, "golden", "tables")


def load_expected():
    with open(os.path.join(HERE, "golden", "expected.json")) as f:
        return json.load(f)


def to_json_rows(rows):
    def enc(x):
        if isinstance(x, bytes):
            return {"b": x.decode("utf-8", "surrogateescape")}
        if isinstance(x, tuple):
            return [enc(v) for v in x]
        return x
    return [enc(r) for r in rows]

"""Helpers to load the committed golden fixtures (tests/golden/*.json)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def prehashed_arrays(name="prehashed.json"):
    v = load(name)
    xy = np.array([list(bytes.fromhex(x["qx"] + x["qy"])) for x in v], dtype=np.uint8)
    e = np.array([list(bytes.fromhex(x["e"])) for x in v], dtype=np.uint8)
    r = np.array([list(bytes.fromhex(x["r"])) for x in v], dtype=np.uint8)
    s = np.array([list(bytes.fromhex(x["s"])) for x in v], dtype=np.uint8)
    exp = np.array([x["expect"] for x in v], dtype=np.int64)
    labels = [x["label"] for x in v]
    return xy, e, r, s, exp, labels

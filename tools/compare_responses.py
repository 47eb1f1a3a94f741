#!/usr/bin/env python3
"""Compare two bench.py --dump-responses files: the same sample ids, and per id the same
token row (e.g. a 2-rank run vs a 1-rank run of the same query).  Prints one JSON line."""
import json
import sys

import numpy as np


def rows(path):
    z = np.load(path)
    ids, lens, toks = z["ids"], z["lens"], z["toks"]
    offs = np.concatenate([[0], np.cumsum(lens)])
    return {int(i): toks[offs[k]: offs[k + 1]] for k, i in enumerate(ids)}


def main(a, b):
    ra, rb = rows(a), rows(b)
    same_ids = set(ra) == set(rb)
    mism = sum(1 for i in ra if i not in rb or not np.array_equal(ra[i], rb[i]))
    out = {"a": a, "b": b, "samples_a": len(ra), "samples_b": len(rb), "same_ids": same_ids,
           "mismatched_rows": mism, "tokens_a": int(sum(len(v) for v in ra.values())),
           "identical": same_ids and mism == 0}
    print(json.dumps(out))
    return 0 if out["identical"] else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))

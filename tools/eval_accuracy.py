#!/usr/bin/env python3
"""Word error rate of a LoadGen accuracy log (the reference's eval_accuracy.py CLI).

    python tools/eval_accuracy.py --log_path mlperf_log_accuracy.json --manifest_path dev-clean-wav.json
Prints "Word Error Rate: X%, accuracy=Y%" and writes hypotheses.log ("i::text" per sample).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rnnt-inference_amd"))

from rnnt_amd import accuracy  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log_path", required=True)
    ap.add_argument("--manifest_path", required=True)
    ap.add_argument("--max_duration", type=float, default=15.0)
    ap.add_argument("--hypotheses", default="hypotheses.log")
    args = ap.parse_args()
    wer, _, _ = accuracy.eval_acc(args.log_path, args.manifest_path, args.max_duration)
    print(f"Word Error Rate: {wer * 100}%, accuracy={(1 - wer) * 100}%")
    hyps = accuracy.read_accuracy_log(args.log_path)
    with open(args.hypotheses, "w") as f:
        for i in sorted(hyps):
            f.write(f"{i}::{accuracy.seq_to_sen(hyps[i])}\n")


if __name__ == "__main__":
    main()

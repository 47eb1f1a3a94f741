"""Accuracy-mode plumbing: the response wire format, transcripts and word error rate.

* Wire format: a response is the sample's int32 labels, ``res_len * 4`` bytes starting at
  ``state.res_[i]`` (QuerySamplesComplete, reference csrc/torch_sut.cpp:221-236); LoadGen's
  accuracy log stores it hex-encoded per sample (``{"qsl_idx", "data"}``) and the checker reads
  it back with ``array("I", bytes.fromhex(data))`` (eval_accuracy.py:91-93).
* ``seq_to_sen``: labels -> text over [' ', a-z, "'"] (models/utils.py:23-57).
* ``word_error_rate``: word-level edit distance summed over utterances / reference words
  (eval_accuracy.py:29-70): ``(wer, errors, words)``, ``inf`` when there are no reference words.
* ``eval_acc``: eval_accuracy.py:78-99 -- manifest transcripts of the samples with
  ``original_duration <= max_duration`` against the logged hypotheses.
"""
import json

import numpy as np

from .config import LABELS


def encode_response(tokens):
    """int32 labels -> the hex payload LoadGen logs for the sample (little-endian int32)."""
    return np.ascontiguousarray(tokens, dtype="<i4").tobytes().hex().upper()


def decode_response(data):
    """hex payload -> labels (the checker's array("I", ...): unsigned 32-bit, little-endian)."""
    return np.frombuffer(bytes.fromhex(data), dtype="<u4").astype(np.int64)


def seq_to_sen(seq, seq_len=None):
    seq = np.asarray(seq)
    n = len(seq) if seq_len is None else int(seq_len)
    return "".join(LABELS[int(t)] for t in seq[:n])


def edit_distance(a, b):
    """Levenshtein distance between two token sequences (one DP row, numpy over the shorter)."""
    if len(a) < len(b):
        a, b = b, a
    if not b:
        return len(a)
    bt = np.asarray(b, dtype=object)
    row = np.arange(len(b) + 1)
    for i, x in enumerate(a, 1):
        sub = row[:-1] + (bt != x)
        nxt = np.empty_like(row)
        nxt[0] = i
        best = np.minimum(sub, row[1:] + 1)  # substitution / match, deletion
        for j in range(1, len(b) + 1):      # insertion runs left to right
            nxt[j] = min(best[j - 1], nxt[j - 1] + 1)
        row = nxt
    return int(row[-1])


def word_error_rate(hypotheses, references):
    if len(hypotheses) != len(references):
        raise ValueError(f"word error rate needs as many hypotheses as references "
                         f"({len(hypotheses)} vs {len(references)})")
    errors = words = 0
    for h, r in zip(hypotheses, references):
        rw = r.split()
        words += len(rw)
        errors += edit_distance(h.split(), rw)
    return (errors / words if words else float("inf")), errors, words


def write_accuracy_log(responses, path):
    """responses: {qsl_idx: int32 labels} -> a LoadGen-style mlperf_log_accuracy.json."""
    entries = [{"seq_id": i, "qsl_idx": int(k), "data": encode_response(v)}
               for i, (k, v) in enumerate(sorted(responses.items()))]
    with open(path, "w") as f:
        json.dump(entries, f)


def read_accuracy_log(path):
    """-> {qsl_idx: labels}."""
    with open(path) as f:
        return {int(e["qsl_idx"]): decode_response(e["data"]) for e in json.load(f)}


def eval_acc(log_path, manifest_path, max_duration=15.0):
    """Word error rate of a LoadGen accuracy log against a LibriSpeech-style manifest."""
    with open(manifest_path) as f:
        manifest = json.load(f)
    refs = [s["transcript"] for s in manifest if s["original_duration"] <= max_duration]
    hyps_by_idx = read_accuracy_log(log_path)
    hyps = [None] * len(hyps_by_idx)
    for k, v in hyps_by_idx.items():
        hyps[k] = seq_to_sen(v)
    return word_error_rate(hyps, refs)

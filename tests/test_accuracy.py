"""Accuracy-mode plumbing (rnnt_amd/accuracy.py): the response wire format read back the way
the reference checker does (array("I", bytes.fromhex(...)), eval_accuracy.py:91-93), the word
error rate (eval_accuracy.py:29-70) against a plain dynamic-programming edit distance, and
eval_acc end to end on a LibriSpeech-style manifest."""
import array
import json

import numpy as np
import pytest

from rnnt_amd import accuracy as A
from rnnt_amd.config import LABELS


def _dp(a, b):
    d = [[0] * (len(b) + 1) for _ in range(len(a) + 1)]
    for i in range(len(a) + 1):
        d[i][0] = i
    for j in range(len(b) + 1):
        d[0][j] = j
    for i in range(1, len(a) + 1):
        for j in range(1, len(b) + 1):
            d[i][j] = min(d[i - 1][j] + 1, d[i][j - 1] + 1, d[i - 1][j - 1] + (a[i - 1] != b[j - 1]))
    return d[-1][-1]


def test_wire_format_roundtrip():
    toks = np.array([0, 1, 27, 5, 26, 13], np.int32)
    data = A.encode_response(toks)
    assert list(array.array("I", bytes.fromhex(data))) == toks.tolist()  # the checker's decode
    np.testing.assert_array_equal(A.decode_response(data), toks)
    assert A.encode_response(np.zeros(0, np.int32)) == ""


@pytest.mark.parametrize("seed", range(6))
def test_edit_distance_matches_dp(seed):
    rng = np.random.default_rng(seed)
    a = list(rng.integers(0, 4, rng.integers(0, 12)))
    b = list(rng.integers(0, 4, rng.integers(0, 12)))
    assert A.edit_distance(a, b) == _dp(a, b) == A.edit_distance(b, a)


def test_word_error_rate():
    assert A.word_error_rate(["a b c"], ["a b d"]) == (1 / 3, 1, 3)
    assert A.word_error_rate(["the cat", "sat"], ["the cat", "sat on"]) == (1 / 4, 1, 4)
    assert A.word_error_rate([""], [""])[0] == float("inf")
    with pytest.raises(ValueError):
        A.word_error_rate(["a"], [])


def test_seq_to_sen_labels():
    assert A.seq_to_sen([8, 9, 0, 27, 19], 5) == "hi 's"
    assert A.seq_to_sen([1, 2, 3], 2) == "ab"
    assert len(LABELS) == 28


def test_eval_acc_end_to_end(tmp_path):
    refs = ["hello world", "a test", "too long to keep"]
    manifest = [{"transcript": refs[0], "original_duration": 3.0},
                {"transcript": refs[1], "original_duration": 15.0},
                {"transcript": refs[2], "original_duration": 16.1}]  # filtered out (> 15 s)
    mp = tmp_path / "manifest.json"
    mp.write_text(json.dumps(manifest))
    enc = {c: i for i, c in enumerate(LABELS)}
    hyps = {0: [enc[c] for c in "hello word"], 1: [enc[c] for c in "a test"]}
    lp = tmp_path / "mlperf_log_accuracy.json"
    A.write_accuracy_log({k: np.array(v, np.int32) for k, v in hyps.items()}, lp)
    wer, errors, words = A.eval_acc(str(lp), str(mp))
    assert (errors, words) == (1, 4) and wer == 0.25


def test_eval_accuracy_cli(tmp_path):
    import subprocess
    import sys
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mp, lp = tmp_path / "m.json", tmp_path / "log.json"
    mp.write_text(json.dumps([{"transcript": "ab c", "original_duration": 2.0}]))
    A.write_accuracy_log({0: np.array([1, 2, 0, 3], np.int32)}, lp)
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "eval_accuracy.py"), "--log_path", str(lp),
                          "--manifest_path", str(mp), "--hypotheses", str(tmp_path / "h.log")],
                         capture_output=True, text=True, check=True).stdout
    assert "Word Error Rate: 0.0%" in out
    assert (tmp_path / "h.log").read_text() == "0::ab c\n"

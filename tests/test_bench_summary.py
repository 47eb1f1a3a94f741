"""bench.py's summary of a measured run on the CPU, in particular a rank whose share of the query is
empty (a query of fewer batches than ranks, or every claim taken by faster ranks): round 5's
multi-rank rehearsal crashed there (np.concatenate of no batches, VERDICT r05 "what's weak" 1)."""
import json
import sys

import numpy as np

import bench


def _args(monkeypatch, *extra):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "2", *extra])
    return bench.parse()


def _stats(enc_ms=0.0, greedy_ms=0.0, jt_ms=0.0, ticks=0):
    return {"encode_ms": enc_ms, "joint_trans_ms": jt_ms, "greedy_ms": greedy_ms, "step_launches": ticks,
            "decode_steps": 0, "encode_calls": 0, "decode_calls": 0}


def test_empty_share(monkeypatch):
    args = _args(monkeypatch)
    lengths = np.array([500, 300, 120], np.int32)
    out = bench.summarize(args, 3, 3 * args.query, 1.5, _stats(), _stats(), lengths, [], None, 0, None)
    json.dumps(out)
    assert out["value"] == round(3 * args.query * 2 / 1.5, 2)
    assert out["roofline"]["achieved"] == 0.0 and out["roofline"]["encode_us_per_tick_events"] is None
    assert out["config"]["batches_run_rank0"] == 0 and out["config"]["encoder_frames_per_query_rank0"] == 0


def test_share_work_counted(monkeypatch):
    args = _args(monkeypatch)
    lengths = np.array([500, 300, 120], np.int32)
    mine = [(np.array([0, 1]), np.array([0, 1])), (np.array([2]), np.array([2]))]
    got = (np.array([0, 1, 2]), np.array([5, 3, 1], np.int32), np.zeros(9, np.int32))
    out = bench.summarize(args, 1, 3, 0.5, _stats(100.0, 40.0, 4.0, 1000), _stats(40.0, 20.0, 2.0, 500),
                          lengths, mine, got, 9, None)
    json.dumps(out)
    from rnnt_amd.config import encoder_frames, encoder_ops
    ops = sum(encoder_ops(int(v)) for v in lengths)
    assert out["roofline"]["achieved"] == round(ops * 2 / 0.1 / 1e12, 2)
    assert out["config"]["encoder_frames_per_query_rank0"] == sum(encoder_frames(int(v)) for v in lengths)
    assert out["config"]["emitted_symbols_per_query"] == 9

"""SUT warmup (OfflineSUT::warmup / ServerSUT::warmup, torch_sut.cpp:124-138, 328-352, over
QSL::GenerateDummySamples, rnnt_qsl.cpp:136-147), host side: every engine runs `iters` dummy
batches of MAX_FEA_LEN-frame N(0,1) samples through encode + decode and nothing is completed.
The device calls are stood in for (the GPU suite runs the real warmup: tests/test_offline_gpu.py)."""
import contextlib

import numpy as np

from rnnt_amd.config import RNNTParam as R
from rnnt_amd.sut import DummyQSL, OfflineSUT, RNNTQSL


class _Eng:
    def __init__(self, device, max_batch):
        self.device, self.max_batch, self.max_res = device, max_batch, 8
        self.calls = []


class _HostSUT(OfflineSUT):
    def _stream_for(self, eng):
        return None

    def _device_scope(self, eng, st):
        return contextlib.nullcontext()

    def _encode(self, eng, st, ids, idx, n, n_pad, qsl=None):
        inp = (qsl or self.qsl_for(eng.device)).batch_inputs(idx, n_pad, "cpu")
        eng.calls.append(("encode", n, n_pad, inp["T"], tuple(inp["store"].shape), inp["lens_host"].copy(),
                          inp["lens"][n:].abs().sum().item(), tuple(inp["offsets"].tolist())))
        return n

    def _decode(self, eng, st, n):
        eng.calls.append(("decode", n))
        return np.zeros(n, np.int32), np.zeros((n, 1), np.int32)


def test_offline_warmup_runs_every_engine_and_completes_nothing():
    qsl = RNNTQSL([None] * 3, np.array([10, 20, 30], np.int32))
    engines = [_Eng(0, 512), _Eng(0, 512), _Eng(1, 100)]
    sut = _HostSUT(engines, qsl, batch_size=300)
    sut.warmup(iters=2)
    for e in engines:
        n = min(300, e.max_batch)
        enc = [c for c in e.calls if c[0] == "encode"]
        assert len(enc) == 2 and [c[0] for c in e.calls] == ["encode", "decode"] * 2
        for c in enc:
            _, nn, n_pad, T, shape, lh, pad_lens, offs = c
            assert nn == n and n_pad % 256 == 0 and n_pad >= n
            # gather form: one MAX_FEA_LEN-frame sample in the store, every row at offset 0
            assert T == R.MAX_FEA_LEN and shape == (R.MAX_FEA_LEN, R.trans_input_size)
            assert np.all(lh == R.MAX_FEA_LEN) and pad_lens == 0 and offs == (0,) * n
    assert sut.take_completed()[0].size == 0 and not sut.responses


def test_dummy_samples_are_seeded_normal_features():
    d = DummyQSL(frames=40, seed=3)
    a = d.batch_inputs(np.zeros(5, np.int64), 256, "cpu")
    b = d.batch_inputs(np.zeros(5, np.int64), 256, "cpu")
    assert a["store"].shape == (40, R.trans_input_size) and a["T"] == 40
    assert a["offsets"].tolist() == [0] * 5 and a["lens"][:5].tolist() == [40] * 5 and int(a["lens"][5:].sum()) == 0
    assert bool((a["store"] == b["store"]).all())  # deterministic
    assert abs(float(a["store"].std()) - 1.0) < 0.05
    assert a["lens"][:5].tolist() == [40] * 5 and int(a["lens"][5:].abs().sum()) == 0

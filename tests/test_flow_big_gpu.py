"""The persistent dataflow encode (lstm_i8_flow_kernel) on batches beyond 256 rows: the 256 x 256
task tile, 256-row batch tiles, tasks of every layer-step dealt from one device queue (development
path, RNNT_ENC_TILE=flow / rnnt_engine_set_tile(e, "flow")).  The int8 encoder is exact, so the
encoder frames must equal the tick path's bit for bit on every valid frame, and the tokens must be
identical; the first rows are checked against the restatement too."""
import numpy as np
import pytest

from rnnt_amd import synthetic

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _valid(f, lens):
    fl = (np.asarray(lens) + 1) // 2
    return np.concatenate([f[: fl[n], n].reshape(-1) for n in range(len(lens))])


def _encode_decode(eng, x, lens, n):
    T = x.shape[0]
    f = torch.zeros(((T + 1) // 2, x.shape[1], 1024), dtype=torch.float32, device="cuda")
    res = torch.empty((n, eng.max_res), dtype=torch.int32, device="cuda")
    rl = torch.empty(n, dtype=torch.int32, device="cuda")
    lp = np.zeros(x.shape[1], np.int32)
    lp[:n] = lens
    eng.encode(torch.from_numpy(x).cuda(), torch.from_numpy(lp).cuda(), lens, n=n, f_out=f)
    eng.decode(res, rl)
    torch.cuda.synchronize()
    return f.cpu().numpy(), res.cpu().numpy(), rl.cpu().numpy()


@pytest.mark.parametrize("n, n_pad", [(1000, 1024), (700, 768)])
def test_big_flow_equals_ticks(n, n_pad, oracle):
    from rnnt_amd import weights
    from rnnt_amd.engine import Engine
    pm, _ = weights.build_model()
    T = 37
    lens = np.sort(np.random.default_rng(n).integers(0, T + 1, n).astype(np.int32))[::-1].copy()
    lens[0] = T
    lp = np.zeros(n_pad, np.int32)
    lp[:n] = lens
    x = synthetic.make_features(T, n_pad, seed=n, lens=lp)
    eng = Engine(pm, device=0, max_batch=n_pad, max_frames=64)
    try:
        out = {}
        for tile in ("auto", "flow", "auto"):  # ticks, flow, ticks again (state reset between calls)
            eng.set_tile(tile)
            out.setdefault(tile, []).append(_encode_decode(eng, x, lens, n))
    finally:
        eng.close()
    (ft, rt, lt), (ft2, rt2, lt2) = out["auto"]
    ff, rf, lf = out["flow"][0]
    np.testing.assert_array_equal(_valid(ff[:, :n], lens).view(np.uint32), _valid(ft[:, :n], lens).view(np.uint32))
    np.testing.assert_array_equal(lf, lt)
    np.testing.assert_array_equal(rf, rt)
    np.testing.assert_array_equal(lt2, lt)
    fo = oracle.encoder_i8(pm, x[:, :8], lp[:8])
    np.testing.assert_array_equal(_valid(ff[:, :8], lens[:8]).view(np.uint32), _valid(fo, lens[:8]).view(np.uint32))

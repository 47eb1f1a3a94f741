"""HIP featurizer (rnnt_featurizer_run) vs the float64 restatement (oracle/featurizer.py).

Tolerance: the GPU computes in fp32 (radix-4 FFT, fp32 mel sums, logf) and the oracle in
float64; normalised features agree to FEAT_TOL absolute (unit-variance features, so this is
also ~relative).  Padding (time past feat_lens, channels 240..255, batch rows past n) and the
lengths are exact.  Rows are independent: a row's features are bit-identical whatever batch it
is in and whether samples come from a zero-padded [N][stride] batch or ragged storage + offsets.
"""
import numpy as np
import pytest

from oracle import featurizer as OF
from rnnt_amd import synthetic

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

FEAT_TOL = 2e-3

# configs/rnnt.toml [input_eval] (the reference's featurizer kwargs; /root/reference is not on the GPU box)
INPUT_EVAL = dict(normalize="per_feature", sample_rate=16000, window_size=0.02, window_stride=0.01, window="hann",
                  features=80, n_fft=512, frame_splicing=3, dither=0.00001, feat_type="logfbank", pad_to=0)

LENS = [0, 1, 100, 257, 479, 480, 16037, 160 * 96 + 5, 96000, 239999, 240000]


@pytest.fixture(scope="module")
def fz():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rnnt_amd.featurizer import AudioProcessing
    proc = AudioProcessing("quant", **INPUT_EVAL)
    yield proc.featurizer
    proc.featurizer.close()


def _batch(wavs):
    n, L = len(wavs), max([len(w) for w in wavs] + [1])
    x = torch.zeros((n, L), dtype=torch.float32)
    for i, w in enumerate(wavs):
        x[i, :len(w)] = w.cpu()
    return x.cuda(), torch.tensor([len(w) for w in wavs], dtype=torch.int32)


def _oracle(fz, wavs, n_pad, T_out):
    return OF.featurize([w.double().numpy() for w in wavs], fz.window, fz.fb, n_pad=n_pad, T_out=T_out,
                        preemph=0.97, dither=1e-5)


def test_gpu_vs_oracle_ragged(fz):
    wavs = synthetic.make_wavs(LENS, seed=21)
    x, lens = _batch(wavs)
    n_pad, T_out = 16, 505
    feats, flen = fz.featurize(x, lens.cuda(), lens.numpy(), n_pad=n_pad, T_out=T_out)
    torch.cuda.synchronize()
    ref, rlen = _oracle(fz, wavs, n_pad, T_out)
    g = feats.cpu().numpy()
    np.testing.assert_array_equal(flen.cpu().numpy(), rlen)
    assert rlen.tolist()[:len(LENS)] == [OF.frames(L)[1] for L in LENS]
    pad = ref == 0.0
    assert np.all(g[pad] == 0.0)  # exact zeros in every padding position
    err = np.abs(g.astype(np.float64) - ref).max()
    assert err <= FEAT_TOL, err
    print("max |gpu - oracle| =", err)


def test_offsets_and_batch_invariance(fz):
    L = [48000, 3200, 0, 777, 150000]
    wavs = synthetic.make_wavs(L, seed=22)
    x, lens = _batch(wavs)
    a, al = fz.featurize(x, lens.cuda(), lens.numpy(), n_pad=8, T_out=320)
    flat = torch.cat([w.cuda() for w in wavs] + [torch.zeros(1, device="cuda")])
    off = torch.tensor(np.concatenate([[0], np.cumsum(L)[:-1]]), dtype=torch.int64, device="cuda")
    b, bl = fz.featurize(flat, lens.cuda(), lens.numpy(), n_pad=8, T_out=320, offsets=off)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.cpu().numpy().view(np.uint32), b.cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(al.cpu().numpy(), bl.cpu().numpy())
    # one row alone (same T_out) == the same row inside the batch
    c, _ = fz.featurize(x[4:5].contiguous(), lens[4:5].cuda(), lens[4:5].numpy(), n_pad=1, T_out=320)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(c.cpu().numpy()[:, 0].view(np.uint32), a.cpu().numpy()[:, 4].view(np.uint32))


def test_ragged_rows_equal_padded_batch(fz):
    """rnnt_featurizer_run_rows (the Server feature store's entry): each sample's frames land as
    240-channel rows at its row offset, bit-identical to its column of the padded batch, and no
    other store row is touched (sentinel)."""
    from rnnt_amd._lib import EngineError
    L = [48000, 3200, 0, 777, 150000, 1]
    wavs = synthetic.make_wavs(L, seed=26)
    flat = torch.cat([w.cuda() for w in wavs] + [torch.zeros(1, device="cuda")])
    off = torch.tensor(np.concatenate([[0], np.cumsum(L)[:-1]]), dtype=torch.int64, device="cuda")
    lens = torch.tensor(L, dtype=torch.int32)
    fr = [OF.frames(v)[1] for v in L]
    a, al = fz.featurize(flat, lens.cuda(), lens.numpy(), n_pad=8, T_out=max(fr), offsets=off)
    store = torch.full((4000, 240), 7.25, device="cuda")
    rows = np.array([3000, 10, 2000, 400, 1000, 3990], np.int64)  # out of order, gaps between
    fl = fz.featurize_rows(flat, lens.cuda(), lens.numpy(), store, rows, max_frames=max(fr), offsets=off)
    torch.cuda.synchronize()
    assert fl.cpu().tolist()[:len(L)] == fr == al.cpu().tolist()[:len(L)]
    s, g = store.cpu().numpy(), a.cpu().numpy()
    used = np.zeros(len(s), bool)
    for i, (r, T) in enumerate(zip(rows, fr)):
        np.testing.assert_array_equal(s[r:r + T].view(np.uint32), g[:T, i, :240].view(np.uint32), err_msg=f"row {i}")
        used[r:r + T] = True
    assert np.all(s[~used] == 7.25)
    with pytest.raises(ValueError, match="outside the store"):
        fz.featurize_rows(flat, lens.cuda(), lens.numpy(), store, rows + 600, max_frames=max(fr), offsets=off)
    with pytest.raises(ValueError, match="max_frames"):
        fz.featurize_rows(flat, lens.cuda(), lens.numpy(), store, rows, max_frames=max(fr) - 1, offsets=off)
    with pytest.raises(EngineError):  # the C ABI's own check
        from rnnt_amd import _lib
        _lib.check(_lib.lib().rnnt_featurizer_run_rows(fz._h, flat.data_ptr(), off.data_ptr(), 0, lens.cuda().data_ptr(),
                                                       lens.numpy().ctypes.data, len(L), store.data_ptr(),
                                                       torch.zeros(len(L), dtype=torch.int64, device="cuda").data_ptr(),
                                                       fl.data_ptr(), max(fr) - 1, None), "run_rows")


def test_forward_mirror_layout(fz):
    wavs = synthetic.make_wavs([16000, 8000, 4000], seed=23)
    x, lens = _batch(wavs)
    y, yl = fz(x, lens, pad_batch_size=True)  # features.py:185-252 signature
    torch.cuda.synchronize()
    T = OF.frames(16000)[1]
    assert tuple(y.shape) == (32, 256, T) and yl.shape[0] == 32
    assert yl.cpu().tolist()[:4] == [T, OF.frames(8000)[1], OF.frames(4000)[1], 0]
    ref, _ = _oracle(fz, wavs, 32, T)
    assert np.abs(y.permute(2, 0, 1).cpu().numpy() - ref).max() <= FEAT_TOL


def test_t_out_too_small_raises(fz):
    from rnnt_amd._lib import EngineError
    wavs = synthetic.make_wavs([240000], seed=24)
    x, lens = _batch(wavs)
    with pytest.raises(EngineError):
        fz.featurize(x, lens.cuda(), lens.numpy(), n_pad=1, T_out=500)  # 15 s = 501 frames


def test_wav_to_tokens_matches_oracle(fz, oracle):
    """featurizer -> int8 engine end to end: tokens identical to the CPU restatement run on the
    GPU features (the encoder/decoder parity of tests/test_gpu_parity.py, fed by the front end)."""
    from rnnt_amd import weights
    from rnnt_amd.engine import Engine
    pm, _ = weights.build_model()
    frames = np.array([60, 41, 17, 3, 1], np.int64)
    L = synthetic.wav_lengths_for_frames(frames, seed=25)
    wavs = synthetic.make_wavs(L, seed=25)
    x, lens = _batch(wavs)
    T, n, n_pad = int(frames.max()), len(L), 256
    feats, flen = fz.featurize(x, lens.cuda(), lens.numpy(), n_pad=n_pad, T_out=T)
    e = Engine(pm, device=0, max_batch=256, max_frames=500)
    try:
        res = torch.empty((n, e.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        fl_host = flen.cpu().numpy()
        e.infer(feats, flen, fl_host[:n], res, rl, n=n)
        torch.cuda.synchronize()
    finally:
        e.close()
    assert fl_host[:n].tolist() == frames.tolist()
    fo = oracle.encoder_i8(pm, np.ascontiguousarray(feats.cpu().numpy()[:, :n]), fl_host[:n])
    ro, rlo, _ = oracle.greedy_decode(pm, fo, (fl_host[:n] + 1) // 2, max_res=res.shape[1])
    np.testing.assert_array_equal(rl.cpu().numpy(), rlo)
    np.testing.assert_array_equal(res.cpu().numpy(), ro)
    assert rlo.sum() > 0


def test_server_sut_over_wav_qsl(oracle):
    """WAV=true Server path: GpuWavQSL featurizes each dynamic batch on the worker's stream while
    the other engine's encode / decode run; every answer -- the Server's and one Offline batch of
    the same audio -- equals the CPU restatement on the same features.  A mismatch names its
    sample, batch, engine, the batch's rows and which side is wrong (round-2 failure: featurizer
    batches corrupted beside a concurrent decode, see test_featurizer_beside_concurrent_decode)."""
    import time
    from rnnt_amd import weights
    from rnnt_amd.engine import Engine
    from rnnt_amd.sut import DynamicBatchServerSUT, GpuWavQSL, QuerySample
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    pm, _ = weights.build_model()
    frames = np.minimum(synthetic.devclean_lengths(24, seed=61), 120)
    wavs = synthetic.make_wavs(synthetic.wav_lengths_for_frames(frames, seed=61), seed=61, device="cuda")
    qsl = GpuWavQSL(wavs)
    assert qsl.lengths.tolist() == frames.tolist()
    n = len(frames)
    x, lens, bl = qsl.assemble(list(range(n)))
    torch.cuda.synchronize()
    feats = np.ascontiguousarray(x.cpu().numpy()[:, :n])
    engines = [Engine(pm, device=0, max_batch=64, max_frames=128) for _ in range(2)]
    try:
        fo = oracle.encoder_i8(pm, feats, bl)
        ro, rlo, _ = oracle.greedy_decode(pm, fo, (bl + 1) // 2, max_res=engines[0].max_res)
        want = [ro[i, : rlo[i]] for i in range(n)]
        assert rlo.sum() > 0
        srv = DynamicBatchServerSUT(engines, qsl, max_batch=8)
        srv.start()
        samples = [QuerySample(id=i, index=i) for i in range(n)]
        for k in range(0, n, 5):
            srv.issue_query(samples[k:k + 5])
            time.sleep(0.002)
        deadline = time.time() + 60
        while len(srv.latency) < n and time.time() < deadline:
            time.sleep(0.01)
        srv.stop()
        assert not srv.errors and len(srv.responses) == n, srv.errors
        res = torch.empty((n, engines[0].max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        engines[0].infer(x, lens, bl, res, rl, n=n)
        res, rl = res.cpu().numpy(), rl.cpu().numpy()
        where = {i: (b, j, ids) for b, (j, ids) in enumerate(srv.batch_log) for i in ids}
        bad = []
        for i in range(n):
            srv_ok = np.array_equal(srv.responses[i], want[i])
            off_ok = np.array_equal(res[i, : rl[i]], want[i])
            if not (srv_ok and off_ok):
                b, j, ids = where[i]
                bad.append(f"sample {i} ({frames[i]} frames): server {'ok' if srv_ok else 'WRONG'} "
                           f"(batch {b} on engine {j}, rows {ids}, {len(srv.responses[i])} vs {len(want[i])} tokens), "
                           f"offline batch {'ok' if off_ok else 'WRONG'}; tick tiles auto (per tick)")
        assert not bad, "\n".join(bad)
    finally:
        for e in engines:
            e.close()


def test_featurizer_beside_concurrent_decode():
    """Regression for the round-2 intermittent Server mismatch: one featurizer batch repeated on
    one stream while another stream runs greedy decodes must equal the quiet result bit for bit.
    Before fz_logmel_kernel owned its CU, ~13 % of such batches had one STFT frame wrong (the
    frames held by lanes 48-63 of a logmel wave, whenever a decode step workgroup shared the CU);
    tools/diag_fz_concurrency.py holds the full experiment."""
    import threading
    import time
    from rnnt_amd import weights
    from rnnt_amd.engine import Engine
    from rnnt_amd.sut import GpuWavQSL
    pm, _ = weights.build_model()
    frames = np.minimum(synthetic.devclean_lengths(24, seed=61), 120)
    qsl = GpuWavQSL(synthetic.make_wavs(synthetic.wav_lengths_for_frames(frames, seed=61), seed=61, device="cuda"))
    idx = list(range(10, 18))
    ref, _, _ = qsl.assemble(idx)
    torch.cuda.synchronize()
    ref = ref[:, :8].cpu().numpy()
    eng = Engine(pm, device=0, max_batch=1024, max_frames=256)
    try:
        lp = np.full(1024, 200, np.int32)
        eng.encode(torch.from_numpy(synthetic.make_features(200, 1024, seed=5)).cuda(), torch.from_numpy(lp).cuda(),
                   lp, n=1024)
        res = torch.empty((1024, eng.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(1024, dtype=torch.int32, device="cuda")
        stop, decodes = threading.Event(), [0]

        def decode_loop():
            st = torch.cuda.Stream()
            while not stop.is_set():
                eng.decode(res, rl, stream=st)
                st.synchronize()
                decodes[0] += 1

        th = threading.Thread(target=decode_loop, daemon=True)
        th.start()
        st = torch.cuda.Stream()
        iters, bad = 0, 0
        t_end = time.time() + 3.0
        try:
            while time.time() < t_end:
                with torch.cuda.stream(st):
                    xb, _, _ = qsl.assemble(idx)
                    got = xb[:, :8].cpu().numpy()
                iters += 1
                bad += int(not np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
        finally:
            stop.set()
            th.join()
        assert decodes[0] >= 2 and iters >= 100, (decodes[0], iters)
        assert bad == 0, f"{bad} of {iters} featurizer batches differ from the quiet result beside {decodes[0]} decodes"
    finally:
        eng.close()


def test_own_cu_switch_same_features(fz, monkeypatch):
    """RNNT_FZ_OWN_CU=1: the round-3 CU-owning LDS request, kept as a runtime fallback
    behind the shipped guard (no packed FP32 in any kernel).  Off by default; on, the logmel launch
    requests the rest of the CU's LDS and the features are bit-identical to the default build's."""
    from rnnt_amd import _lib
    from rnnt_amd.featurizer import AudioProcessing
    assert _lib.lib().rnnt_featurizer_own_cu_lds(fz._h) == 0
    monkeypatch.setenv("RNNT_FZ_OWN_CU", "1")
    own = AudioProcessing("quant", **INPUT_EVAL).featurizer
    try:
        assert _lib.lib().rnnt_featurizer_own_cu_lds(own._h) > 0
        wavs = synthetic.make_wavs(LENS, seed=23)
        x, lens = _batch(wavs)
        a, la = fz.featurize(x, lens.cuda(), lens.numpy(), n_pad=16, T_out=505)
        b, lb = own.featurize(x, lens.cuda(), lens.numpy(), n_pad=16, T_out=505)
        torch.cuda.synchronize()
        assert torch.equal(la, lb)
        assert np.array_equal(a.cpu().numpy().view(np.uint32), b.cpu().numpy().view(np.uint32))
    finally:
        own.close()

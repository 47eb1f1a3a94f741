"""The compiled TorchModel replacement (rnnt-inference_amd/csrc/sut/rnnt_model_mi355x.hpp, INTEGRATION.md
section 1) driven through the reference SUT's own State protocol.

The harness (csrc/sut/sut_harness.cpp, built by the Makefile against include/rnnt_mi355x.h and libtorch)
runs the model the way the reference's SUT runs TorchModel, with State / PipelineState restated from
metadata.cpp (csrc/sut/sut_state.hpp):
* Offline (OfflineSUT::thInstance, torch_sut.cpp:140-236): several instances at once, instance i calling
  with which = i & 1, each its own State(batch, split_len); split_len > 0 goes through State::next()
  exactly as the reference's run.sh Offline setting (LEN=2, INTER=28, run.sh:68-71).
* Server (ServerSUT::thConsumer, :470-571): consumers with a PipelineState each -- slot refill, chunked
  next(), answers for finished slots only.
Checked: every sample answered once; each payload equals the CPU restatement's tokens; the harness
checks the SOS (-1) fill of res_ past each answered row and res_idx_ = length - 1."""
import json
import os
import subprocess

import numpy as np
import pytest

from rnnt_amd import synthetic, weights

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(REPO, "rnnt-inference_amd", "rnnt_amd", "rnnt_sut_harness")


def _responses(path):
    b = open(path, "rb").read()
    out, off = {}, 0
    while off < len(b):
        sid, size = np.frombuffer(b, np.int32, 2, off)
        off += 8
        assert int(sid) not in out, f"sample {sid} answered twice"
        out[int(sid)] = np.frombuffer(b, np.int32, int(size) // 4, off).copy()
        off += int(size)
    return out


@pytest.fixture(scope="module")
def setup(tmp_path_factory, oracle):
    tmp = tmp_path_factory.mktemp("harness")
    pm, _ = weights.build_model()
    eng_file = weights.save_engine_file(pm, str(tmp / "rnnt.engine"))
    rng = np.random.default_rng(61)
    lens = rng.integers(1, 62, 40).astype(np.int32)
    lens[[3, 17]] = [0, 61]
    lens[[5, 9, 22]] = [1, 2, 33]
    N, T = len(lens), int(lens.max())
    x = synthetic.make_features(T, N, seed=24, lens=lens)[:, :, :240]  # [T][N][240]
    ragged = np.concatenate([x[: lens[i], i] for i in range(N)])  # the QSL's frames back to back
    ragged.astype(np.float32).tofile(tmp / "feats.bin")
    lens.tofile(tmp / "lens.bin")
    fo = oracle.encoder_i8(pm, np.pad(x, ((0, 0), (0, 0), (0, 16))), lens)
    ro, rlo, _ = oracle.greedy_decode(pm, fo, (lens + 1) // 2, max_res=(500 // 2) * 30)
    assert rlo.max() > 3 and rlo[3] == 0
    return dict(tmp=tmp, eng=eng_file, lens=lens, want=[ro[i, : rlo[i]] for i in range(N)])


def _run(setup, name, env_extra=None, **kw):
    tmp = setup["tmp"]
    out = tmp / f"{name}.bin"
    cmd = [HARNESS, "--engine", setup["eng"], "--feats", str(tmp / "feats.bin"), "--lens", str(tmp / "lens.bin"),
           "--out", str(out)]
    for k, v in kw.items():
        cmd += ["--" + k.replace("_", "-"), str(v)]
    env = dict(os.environ, **(env_extra or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["bad_sos_fill_rows"] == 0 and summary["bad_res_idx_rows"] == 0, summary
    return summary, _responses(out)


@pytest.mark.parametrize("threads,split_len,env", [
    (1, -1, {}),                                 # one instance, whole batches
    (3, -1, {"pinned": 1}),                      # batches assembled in pinned memory: DMA'd as they are
    (8, 2, {}),                                  # run.sh's Offline shape: split_len 2, which = index & 1
    (4, 2, {"RNNT_ENGINES_PER_GPU": "1"}),       # more instances than engines: leases wait and are reused
    (6, 4, {"RNNT_ENCODE_TURNS": "0"}),          # encoders of one GPU overlapping
    (8, 2, {"RNNT_GPUS": "0,0"}),                # two GPU pools (both on device 0): which = 0 / 1 -> one each
])
def test_offline_state_protocol(setup, threads, split_len, env):
    assert os.path.exists(HARNESS), "harness not built (make -C rnnt-inference_amd/csrc)"
    N = len(setup["lens"])
    env = dict(env)
    pinned = env.pop("pinned", 0)
    summary, got = _run(setup, f"off_{threads}_{split_len}_{pinned}", env, scenario="offline", threads=threads, batch=6,
                        split_len=split_len, warmup=1 if threads == 8 else 0, intra=2, pinned=pinned)
    assert summary["model_host_seconds"]["dense_pinned_calls"] == (summary["batches"] if pinned else 0), summary
    assert summary["responses"] == N and summary["batches"] == -(-N // 6), summary
    assert sorted(got) == list(range(N))
    for i in range(N):
        np.testing.assert_array_equal(got[i], setup["want"][i], err_msg=f"sample {i}")
    if "RNNT_ENGINES_PER_GPU" in env:
        assert summary["engines_per_gpu"] == [1], summary
    if "RNNT_GPUS" in env:  # the socket's half of the node's GPUs: both pools served batches
        assert len(summary["engines_per_gpu"]) == 2 and min(summary["engines_per_gpu"]) > 0, summary


def test_offline_odd_split_rejected(setup):
    tmp = setup["tmp"]
    r = subprocess.run([HARNESS, "--engine", setup["eng"], "--feats", str(tmp / "feats.bin"), "--lens",
                        str(tmp / "lens.bin"), "--out", str(tmp / "odd.bin"), "--split-len", "3"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "odd split_len" in r.stderr, r.stderr[-2000:]


@pytest.mark.parametrize("threads,batch,split_len,response", [(1, 8, 8, 3), (3, 6, 8, 1), (2, 16, 2, 16)])
def test_server_pipeline_state(setup, threads, batch, split_len, response):
    """PipelineState slots refilled as they finish, each consumer keeping its engine; zero-length samples
    are never answered by the reference's Server (F_lens_ > 0, torch_sut.cpp:552), so the query leaves
    them out."""
    lens = setup["lens"]
    query = np.array([i for i in range(len(lens)) if lens[i] > 0], np.int32)
    qf = setup["tmp"] / "query_server.bin"
    query.tofile(qf)
    summary, got = _run(setup, f"srv_{threads}_{batch}_{split_len}", scenario="server", threads=threads,
                        batch=batch, split_len=split_len, response=response, pro_batch=4, query=qf, intra=2)
    assert summary["responses"] == len(query), summary
    assert sorted(got) == list(range(len(query)))
    for pos, i in enumerate(query):
        np.testing.assert_array_equal(got[pos], setup["want"][i], err_msg=f"query position {pos} (sample {i})")
    assert summary["engines_per_gpu"][0] >= threads


@pytest.fixture(scope="module")
def wav_setup(tmp_path_factory, oracle):
    """WAV=true (launch_sut.sh:53-55): 16 kHz audio, the processor file, and the expected tokens -- the
    CPU restatement of the model on the features the GPU featurizer makes of each utterance (the same
    kernels the AudioProcessor drop-in runs; features are per utterance, so batching does not change them)."""
    import torch
    from rnnt_amd.featurizer import write_processor_file
    from rnnt_amd.sut import GpuWavQSL
    tmp = tmp_path_factory.mktemp("harness_wav")
    pm, _ = weights.build_model()
    eng_file = weights.save_engine_file(pm, str(tmp / "rnnt.engine"))
    proc_file = write_processor_file(str(tmp / "rnnt.processor"))
    frames = np.random.default_rng(81).integers(8, 90, 26).astype(np.int64)
    wav_lens = synthetic.wav_lengths_for_frames(frames, seed=81)
    wavs = synthetic.make_wavs(wav_lens, seed=81)
    np.concatenate([w.numpy() for w in wavs]).astype(np.float32).tofile(tmp / "wav.bin")
    wav_lens.astype(np.int32).tofile(tmp / "wav_lens.bin")
    q = GpuWavQSL([w.cuda() for w in wavs])
    idx = list(range(len(wavs)))
    x, _, bl = q.assemble(idx)
    feats = np.ascontiguousarray(x.cpu().numpy()[:, : len(idx)])
    fo = oracle.encoder_i8(pm, feats, bl)
    ro, rlo, _ = oracle.greedy_decode(pm, fo, (bl + 1) // 2, max_res=250 * 30)
    assert rlo.max() > 3
    torch.cuda.synchronize()
    return dict(tmp=tmp, eng=eng_file, proc=proc_file, want=[ro[i, : rlo[i]] for i in idx])


@pytest.mark.parametrize("scenario,threads,batch,split_len", [("offline", 4, 8, 2), ("offline", 2, 8, -1),
                                                              ("server", 2, 8, 8)])
def test_wav_processor_drop_in(wav_setup, scenario, threads, batch, split_len):
    """The AudioProcessor drop-in (csrc/sut/rnnt_processor_mi355x.hpp) featurizes each batch on the GPU
    and hands the SUT [N_out][256][T] features (a view of pinned memory the model DMAs as it is); every
    payload equals the restatement on the GPU featurizer's features."""
    s = wav_setup
    tmp = s["tmp"]
    out = tmp / f"wav_{scenario}_{threads}_{split_len}.bin"
    cmd = [HARNESS, "--engine", s["eng"], "--processor", s["proc"], "--wav", str(tmp / "wav.bin"), "--wav-lens",
           str(tmp / "wav_lens.bin"), "--out", str(out), "--scenario", scenario, "--threads", str(threads),
           "--batch", str(batch), "--split-len", str(split_len), "--intra", "2", "--warmup", "0"]
    if scenario == "server":
        cmd += ["--response", "2", "--pro-batch", "4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["bad_res_idx_rows"] == 0 and summary["responses"] == len(s["want"]), summary
    if scenario == "offline" and split_len < 0:
        assert summary["model_host_seconds"]["dense_pinned_calls"] == summary["batches"], summary
    got = _responses(out)
    for i, w in enumerate(s["want"]):
        np.testing.assert_array_equal(got[i], w, err_msg=f"sample {i}")

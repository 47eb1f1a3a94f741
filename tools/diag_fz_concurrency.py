"""Diagnostic: is a featurizer batch corrupted while another thread's kernels share the GPU?

Thread A featurizes the same 8 utterances over and over on its own stream and compares every
output bit-for-bit with the first (quiet) result; thread B runs one kind of concurrent work on
its own stream.  Each mode runs for --seconds; per mode the number of corrupted batches and the
(spliced row, channel group) of the corrupted values are reported.

python tools/diag_fz_concurrency.py [--seconds 10] [--modes none,featurize,encode,decode,copy]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--modes", default="none,featurize,encode,decode,copy")
    ap.add_argument("--out", default="gpurun_out/diag_fz.json")
    ap.add_argument("--dump", action="store_true", help="lib built with -DRNNT_DIAG_FZ_DUMP: compare power rows too")
    ap.add_argument("--victim", default="featurize", choices=["featurize", "encode"],
                    help="what thread A repeats and checks: the featurizer batch, or a small-batch int8 encode "
                         "(mini / tiny tick tiles, which can share a CU with the decode kernels)")
    args = ap.parse_args()
    import torch
    from rnnt_amd import synthetic, weights
    from rnnt_amd.engine import Engine
    from rnnt_amd.sut import GpuWavQSL

    frames = np.minimum(synthetic.devclean_lengths(24, seed=61), 120)
    wavs = synthetic.make_wavs(synthetic.wav_lengths_for_frames(frames, seed=61), seed=61, device="cuda")
    qsl = GpuWavQSL(wavs)
    idx = list(range(10, 18))
    ref, _, bl = qsl.assemble(idx)
    torch.cuda.synchronize()
    ref = ref[:, :8].cpu().numpy()
    if args.dump:
        import ctypes as C
        from rnnt_amd import _lib
        dlib = _lib.lib()
        dlib.rnnt_dev_fz_dump.argtypes = [C.c_void_p, C.c_int]
        nch = int(sum((1 + qsl.wav_lengths[i] // 160 + 15) // 16 for i in idx))
        pref = np.zeros((nch, 16, 260), np.float32)
        dlib.rnnt_dev_fz_dump(pref.ctypes.data, nch)
        pbuf = np.zeros_like(pref)
    pm, _ = weights.build_model()
    eng = Engine(pm, device=0, max_batch=1024, max_frames=500)
    feats_b = torch.from_numpy(synthetic.make_features(200, 1024, seed=5)).cuda()
    lens_b = torch.full((1024,), 200, dtype=torch.int32, device="cuda")
    lh = np.full(1024, 200, np.int32)
    res = torch.empty((1024, eng.max_res), dtype=torch.int32, device="cuda")
    rl = torch.empty(1024, dtype=torch.int32, device="cuda")
    eng.encode(feats_b, lens_b, lh, n=1024)
    eng.decode(res, rl)
    torch.cuda.synchronize()
    res_ref, rl_ref = res.cpu().numpy(), rl.cpu().numpy()
    dec_bad = [0]
    if args.victim == "encode":  # 40 rows x 120 frames: one batch tile -> mini / tiny tick tiles
        veng = Engine(pm, device=0, max_batch=256, max_frames=128)
        vn = 40
        vlh = np.full(vn, 120, np.int32)
        vlp = np.zeros(256, np.int32)
        vlp[:vn] = vlh
        vx = torch.from_numpy(synthetic.make_features(120, 256, seed=9, lens=vlp)).cuda()
        vlens = torch.from_numpy(vlp).cuda()
        vf = torch.zeros((60, 256, 1024), dtype=torch.float32, device="cuda")
        veng.encode(vx, vlens, vlh, n=vn, f_out=vf)
        torch.cuda.synchronize()
        vref = vf.cpu().numpy()
    big_a = torch.randn(64 << 20, device="cuda")
    big_b = torch.empty_like(big_a)
    summary = {}
    import ctypes as C
    plib = None
    if any(m.startswith("stress") for m in args.modes.split(",")):
        plib = C.CDLL(os.path.join(REPO, "build_dev", "libprobe_stress.so"))
        plib.probe_stress.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    for mode in args.modes.split(","):
        stop = threading.Event()
        counts = dict(b_iters=0)

        def other():
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                while not stop.is_set():
                    if mode == "featurize":
                        qsl.assemble(list(range(0, 8)))
                    elif mode == "encode":
                        eng.encode(feats_b, lens_b, lh, n=1024, stream=st)
                    elif mode == "decode":
                        eng.decode(res, rl, stream=st)
                    elif mode == "decode_check":  # is the decode itself corrupted beside the featurizer?
                        eng.decode(res, rl, stream=st)
                        st.synchronize()
                        if not (np.array_equal(rl.cpu().numpy(), rl_ref) and np.array_equal(res.cpu().numpy(), res_ref)):
                            dec_bad[0] += 1
                    elif mode.startswith("stress"):  # stress<kind>: synthetic co-runner (tools/probe/probe_stress.hip)
                        kind = int(mode[6:])
                        plib.probe_stress(kind, 2048, {0: 0, 1: 64, 2: 256, 3: 2048, 4: 256}[kind], 20,
                                          C.c_void_p(st.cuda_stream))
                    elif mode == "copy":
                        big_b.copy_(big_a)
                    else:
                        time.sleep(0.01)
                    st.synchronize()
                    counts["b_iters"] += 1

        th = threading.Thread(target=other, daemon=True)
        th.start()
        st = torch.cuda.Stream()
        bad, iters, where = 0, 0, []
        t_end = time.time() + args.seconds
        while time.time() < t_end:
            if args.victim == "encode":
                with torch.cuda.stream(st):
                    veng.encode(vx, vlens, vlh, n=vn, f_out=vf, stream=st)
                    fa = vf.cpu().numpy()
                iters += 1
                if not np.array_equal(fa.view(np.uint32), vref.view(np.uint32)):
                    bad += 1
                    dd = np.nonzero(np.any(fa.view(np.uint32) != vref.view(np.uint32), axis=2))
                    where.append(dict(iter=iters, frames=sorted(set(dd[0].tolist()))[:10],
                                      rows=sorted(set(dd[1].tolist()))[:10]))
                continue
            with torch.cuda.stream(st):
                x, _, _ = qsl.assemble(idx)
                xa = x[:, :8].cpu().numpy()
            iters += 1
            d = xa.view(np.uint32) != ref.view(np.uint32)
            if d.any():
                bad += 1
                if args.dump:
                    dlib.rnnt_dev_fz_dump(pbuf.ctypes.data, nch)
                    pd = pbuf.view(np.uint32) != pref.view(np.uint32)
                    for ch, fr in zip(*np.nonzero(pd.any(axis=2))):
                        bins = np.nonzero(pd[ch, fr])[0]
                        where.append(dict(iter=iters, chunk=int(ch), frame=int(fr), nbins=int(len(bins)),
                                          bins=bins[:24].tolist(), lanes=sorted(set(int(b) % 16 for b in bins)),
                                          qs=sorted(set(int(b) // 16 for b in bins))))
                rows = np.nonzero(d.any(axis=(0, 2)))[0]
                for r in rows[:4]:
                    # normalisation spreads one corrupted STFT frame over its channels' every row: find
                    # the (row, 80-channel group) whose error dominates
                    e = np.abs(xa[:, r] - ref[:, r])
                    t, c = np.unravel_index(int(np.argmax(e)), e.shape)
                    where.append(dict(iter=iters, row=int(r), spliced_row=int(t), group=int(c // 80),
                                      stft_frame=int(3 * t + c // 80), in_chunk=int((3 * t + c // 80) % 16),
                                      max_err=float(e.max())))
        stop.set()
        th.join()
        summary[mode] = dict(iters=iters, bad=bad, b_iters=counts["b_iters"], where=where[:40], decode_bad=dec_bad[0])
        print(f"[{mode}] featurize iters {iters}, corrupted {bad}, other-thread iters {counts['b_iters']}, "
              f"decode results wrong {dec_bad[0]}", flush=True)
        dec_bad[0] = 0
        for w in where[:6]:
            print("   ", w, flush=True)
    eng.close()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Featurizer kernels on the host emulation with poisoned LDS (tools/emu/fz_emu.cpp).

Runs the same batch with every fz_logmel workgroup's LDS filled with quiet NaNs, 1e38, zeros and
random bits at workgroup start; the outputs must be bit-identical across poisons (no LDS word is
read before its workgroup wrote it), every element must be written (the output buffer starts as
0xA5 bytes), and the features must match the float64 restatement (oracle/featurizer.py) within
the GPU tests' tolerance.  Lanes of a wave are not in lockstep in the emulation, so an intra-wave
hand-off that relied on lockstep instead of wave_lds_sync would show up here too.

    bash tools/emu/build_fz.sh && python3 tools/emu/fz_emu_check.py [--n 5] [--seed 3]
"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "rnnt-inference_amd"))
sys.path.insert(0, ROOT)

from oracle import featurizer as ofz  # noqa: E402  (test infrastructure: the checker)
from rnnt_amd import synthetic  # noqa: E402
from rnnt_amd.featurizer import make_window, mel_filterbank  # noqa: E402


def run(exe, inp, poison):
    out = inp + "." + poison + ".out"
    env = dict(os.environ, EMU_POISON=poison, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe, inp, out], env=env, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(f"fz_emu ({poison}) failed rc={r.returncode}:\n{r.stderr[-3000:]}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--exe", default=os.path.join(ROOT, "build_dev", "emu_fz", "fz_emu"))
    args = ap.parse_args()
    # ragged lengths incl. a 1-sample row, a row shorter than the reflect pad and chunk-boundary cases
    base = [8000, 3001, 1, 200, 160 * 48 + 37]
    lens = np.array((base * ((args.n + len(base) - 1) // len(base)))[: args.n], np.int64)
    wavs = [w.double().numpy() if hasattr(w, "double") else np.asarray(w, np.float64)
            for w in synthetic.make_wavs(lens.tolist(), seed=args.seed)]
    window, fb = make_window("hann", 320), mel_filterbank(16000, 512, 80)
    n = len(wavs)
    n_pad = (n + 7) // 8 * 8 + 1  # padding rows (and an odd count) must come out zero
    T_out = max(ofz.frames(len(w))[1] for w in wavs)
    maxl = int(lens.max())
    wav = np.zeros((n, maxl), np.float32)
    for i, w in enumerate(wavs):
        wav[i, : len(w)] = w
    with tempfile.TemporaryDirectory() as td:
        inp = os.path.join(td, "in.bin")
        with open(inp, "wb") as f:
            np.array([n, n_pad, T_out], np.int32).tofile(f)
            np.asarray(window, np.float32).tofile(f)
            np.asarray(fb, np.float32).tofile(f)
            lens.astype(np.int32).tofile(f)
            wav.tofile(f)
        outs = {}
        for p in ("nan", "big", "zero", "rand"):
            o = np.fromfile(run(args.exe, inp, p), np.uint8)
            outs[p] = o
            print(f"poison {p}: {o.size} bytes", flush=True)
    ref = outs["nan"]
    same = {p: bool(np.array_equal(o, ref)) for p, o in outs.items()}
    fl = ref[: 4 * n_pad].view(np.int32)
    feats = ref[4 * n_pad:].view(np.float32).reshape(T_out, n_pad, 256)
    want, wl = ofz.featurize([w for w in wavs], window.astype(np.float64), fb.astype(np.float64), n_pad=n_pad,
                             T_out=T_out)
    unwritten = int((ref[4 * n_pad:].view(np.uint32) == 0xA5A5A5A5).sum())
    err = float(np.abs(feats - want).max())
    print({"poisons_bit_identical": same, "lens_equal": bool(np.array_equal(fl, wl)), "unwritten_words": unwritten,
           "max_abs_err_vs_float64": err})
    ok = all(same.values()) and np.array_equal(fl, wl) and unwritten == 0 and err <= 2e-3
    print("OK" if ok else "FAIL")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())

"""Co-residency probe (development tool): encode one 6144-row batch of the bench query alone, then
with a slim kernel (probe_coresident.hip: 4-wave workgroups, 12 VGPRs, 8 KiB LDS -- small enough to
fit beside a 256x256 tick workgroup on its CU) streaming an L2-sized buffer on a second stream.
If the slim workgroups share CUs with the ticks, the encode slows only by what they take from the
CU's issue and load path; if they displace ticks, by their whole CU time.

    hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/coresident/probe_coresident.hip \
        -o tools/coresident/libprobe_coresident.so
    python tools/coresident/run.py   (on a GPU box; prints one JSON line)
"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from rnnt_amd import dist, weights  # noqa: E402
from rnnt_amd.engine import Engine, pad_batch  # noqa: E402
from rnnt_amd.sut import make_batches  # noqa: E402


def main():
    torch.cuda.set_device(0)
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe_coresident.so"))
    lib.probe_slim_launch.restype = C.c_int
    lib.probe_slim_launch.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    pm, _ = weights.build_model()
    qsl = bench.build_qsl(2513, seed=4, device="cuda:0")
    ids, idx = dist.query_arrays(2513, 24576)
    bids, bidx = make_batches(qsl, ids, idx, 6144)[1]
    n = len(bids)
    eng = Engine(pm, device=0, max_batch=6144, max_frames=500)
    se, sp = torch.cuda.Stream(), torch.cuda.Stream()
    b = qsl.batch_inputs(bidx, pad_batch(n), torch.device("cuda", 0))
    buf = torch.ones(int(os.environ.get("PROBE_BYTES", str(2 << 20))) // 4, dtype=torch.float32, device="cuda")
    out = torch.empty(4096 * 256, dtype=torch.float32, device="cuda")

    def encode():
        eng.encode_gather(b["store"], b["offsets"], b["lens"], b["lens_host"], b["T"], n, pad_batch(n), stream=se)

    def probe(iters, grid):
        rc = lib.probe_slim_launch(C.c_void_p(buf.data_ptr()), buf.numel() * 4, iters, grid,
                                   C.c_void_p(out.data_ptr()), C.c_void_p(sp.cuda_stream))
        assert rc == 0

    def timed(fn, st):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        return e0, e1

    res = {"batch_rows": n, "frames": int(b["T"])}
    encode()
    torch.cuda.synchronize()
    enc_alone = []
    for _ in range(3):
        e0, e1 = timed(encode, se)
        torch.cuda.synchronize()
        enc_alone.append(e0.elapsed_time(e1))
    res["encode_alone_ms"] = [round(x, 2) for x in enc_alone]
    target = min(enc_alone) * 0.9
    for grid in (256, 1024):
        e0, e1 = timed(lambda: probe(2000, grid), sp)
        torch.cuda.synchronize()
        per_iter = e0.elapsed_time(e1) / 2000
        iters = max(100, int(target / per_iter))
        p0, p1 = timed(lambda: probe(iters, grid), sp)
        torch.cuda.synchronize()
        alone = p0.elapsed_time(p1)
        runs = []
        for _ in range(3):
            p0, p1 = timed(lambda: probe(iters, grid), sp)
            e0, e1 = timed(encode, se)
            torch.cuda.synchronize()
            runs.append((round(e0.elapsed_time(e1), 2), round(p0.elapsed_time(p1), 2)))
        res[f"grid{grid}"] = {"iters": iters, "probe_alone_ms": round(alone, 2), "encode_ms_with_probe": [r[0] for r in runs],
                              "probe_ms_with_encode": [r[1] for r in runs]}
    eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

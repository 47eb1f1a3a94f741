"""Why does the greedy decode slow down beside an encoder?  (measurement tooling)

Runs on one GPU with two engines: A encodes batch 0 (then decodes it: its decode is what we
time), B encodes batch 1 concurrently.  Cases:
  enc_full / enc_half   encode alone on a full / half-CU-masked stream (checks CU masking works)
  dec_alone             A's decode with nothing beside it
  dec_beside[_rN]       A's decode while B encodes (B's stream keeps N CUs per XCD free)
  dec_only_reserved_rN  A's decode on a stream restricted to the N reserved CUs per XCD
"""
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from rnnt_amd import weights  # noqa: E402
from rnnt_amd.engine import Engine, PartitionedStream, cu_mask_words  # noqa: E402


def main():
    torch.cuda.set_device(0)
    pm, _ = weights.build_model()
    qsl = bench.build_qsl(2513, seed=4)
    batches = bench.make_batches(qsl, 16384, 8192)
    A = Engine(pm, device=0, max_batch=8192, max_frames=500)
    B = Engine(pm, device=0, max_batch=8192, max_frames=500)
    for b in batches:
        b["res"] = torch.empty((b["n"], A.max_res), dtype=torch.int32, device="cuda")
        b["rl"] = torch.empty(b["n"], dtype=torch.int32, device="cuda")
    b0, b1 = batches
    full = PartitionedStream(0)
    out = {}

    def t_enc(eng, b, st):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.encode(b["x"], b["lens"], b["lens_host"], n=b["n"], stream=st)
        st.synchronize()
        return (time.perf_counter() - t0) * 1e3

    t_enc(A, b0, full.stream)
    out["enc_full_ms"] = t_enc(A, b0, full.stream)
    half = PartitionedStream(0, cu_mask_words(16))
    out["enc_half_ms"] = t_enc(A, b0, half.stream)
    half.close()

    def t_dec(st):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        A.decode(b0["res"], b0["rl"], stream=st)
        st.synchronize()
        return (time.perf_counter() - t0) * 1e3

    t_enc(A, b0, full.stream)
    out["dec_alone_ms"] = t_dec(full.stream)

    def beside(dec_stream, enc_mask):
        es = PartitionedStream(0, enc_mask)
        t_enc(A, b0, full.stream)
        res = {}

        def enc_b():
            t0 = time.perf_counter()
            B.encode(b1["x"], b1["lens"], b1["lens_host"], n=b1["n"], stream=es.stream)
            es.stream.synchronize()
            res["enc_ms"] = (time.perf_counter() - t0) * 1e3

        th = threading.Thread(target=enc_b)
        th.start()
        time.sleep(0.005)
        res["dec_ms"] = t_dec(dec_stream)
        th.join()
        es.close()
        return res

    out["dec_beside_r0"] = beside(full.stream, None)
    for r in (2, 4, 8):
        out[f"dec_beside_r{r}"] = beside(full.stream, cu_mask_words(r))
        rs = PartitionedStream(0, cu_mask_words(r, reserved=True))
        t_enc(A, b0, full.stream)
        out[f"dec_only_reserved_r{r}_alone_ms"] = t_dec(rs.stream)
        out[f"dec_only_reserved_r{r}_beside"] = beside(rs.stream, cu_mask_words(r))
        rs.close()
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else {a: round(c, 2) for a, c in v.items()})
                      for k, v in out.items()}, indent=1))
    full.close()
    A.close()
    B.close()


if __name__ == "__main__":
    main()

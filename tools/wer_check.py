"""Development check of bench.py's wer_vs_fp32 sample: GPU int8+bf16 tokens vs the CPU
restatement on the same planted utterances, and the int8-vs-fp32 disagreement split into its
encoder and decoder parts (oracle: int8 / fp32 encoder, each through the bf16 decoder)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle  # noqa: E402
from rnnt_amd import accuracy, planted, synthetic, weights  # noqa: E402
from rnnt_amd.decoder import GreedyDecoder  # noqa: E402
from rnnt_amd.model import RNNT  # noqa: E402

n, seed = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 44
ckpt, task = planted.make_planted_checkpoint()
lens = synthetic.devclean_lengths(n, seed=seed)
feats, truth = planted.planted_features(task, lens, seed=seed + 1)
x = np.zeros((int(lens.max()), n, 240), np.float32)
for i, fe in enumerate(feats):
    x[: len(fe), i] = fe
amax = weights.calibrate_amax(weights.migrate_state_dict(ckpt), x[:, :8], lens[:8])
xd, ld = torch.from_numpy(x).cuda(), torch.from_numpy(lens)
out = {}
hyp = {}
for mode in ("quant", "f32"):
    m = RNNT(ckpt, mode, enable_bf16=(mode == "quant"), amax=amax)
    dec = GreedyDecoder(m, mode, mode == "quant", batch_size=n, device=0)
    res, rl = dec(xd, ld)
    hyp[mode] = (res.cpu().numpy(), rl.cpu().numpy())
    dec.close()
sen = lambda r: [accuracy.seq_to_sen(r[0][i], r[1][i]) for i in range(n)]  # noqa: E731
out["gpu_int8bf16_vs_gpu_f32"] = accuracy.word_error_rate(sen(hyp["quant"]), sen(hyp["f32"]))
mq = RNNT(ckpt, "quant", enable_bf16=True, amax=amax)
m32 = RNNT(ckpt, "f32", enable_bf16=False, amax=amax)
xp = np.zeros((x.shape[0], n, 256), np.float32)
xp[:, :, :240] = x
fi8 = oracle.encoder_i8(mq.pm, xp, lens)
fl = (lens + 1) // 2
r1, l1, _ = oracle.greedy_decode(mq.pm, fi8, fl, max_res=hyp["quant"][0].shape[1])
rows_bad = [i for i in range(n) if l1[i] != hyp["quant"][1][i] or not np.array_equal(r1[i, :l1[i]], hyp["quant"][0][i, :l1[i]])]
out["gpu_vs_oracle_int8bf16_mismatched_rows"] = rows_bad[:20]
out["gpu_vs_oracle_int8bf16_mismatch_count"] = len(rows_bad)
f32 = oracle.encoder_f32(m32.f32_encoder_layers(), x, lens)
r2, l2, _ = oracle.greedy_decode(mq.pm, f32, fl)
out["oracle_int8enc_vs_f32enc_same_bf16_decoder"] = accuracy.word_error_rate(sen((r1, l1)), sen((r2, l2)))
out["oracle_f32enc_bf16dec_vs_gpu_f32"] = accuracy.word_error_rate(sen((r2, l2)), sen(hyp["f32"]))
print(json.dumps(out))

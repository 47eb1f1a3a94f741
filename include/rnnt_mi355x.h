/*
 * rnnt_mi355x.h -- C ABI of the MI355X RNN-T inference engine (librnnt_mi355x.so).
 *
 * The drop-in boundary for the reference's hot path:
 *   - rnnt_engine_encode / rnnt_engine_decode replace the bodies of
 *     TorchModel::encode / TorchModel::decode (reference csrc/rnnt_model.hpp:62-90, 92-124),
 *     called per batch by OfflineSUT::thInstance (csrc/torch_sut.cpp:208-212) and
 *     ServerSUT::thConsumer (:529-531).  Results use the State::res_ / res_idx_ contract
 *     (csrc/metadata.hpp:58-59, metadata.cpp:59-60): res [N][max_res] int32 filled with
 *     SOS (-1), res_len[n] = res_idx_[n] + 1, read by QuerySamplesComplete (torch_sut.cpp:221-236).
 *   - rnnt_engine_infer = encode + decode (TorchModel::forward, rnnt_model.hpp:56-60).
 *   - the rnnt_op_* entry points back the torch.ops.intel_mlperf operator names the reference
 *     TorchScript graph binds to (models/_C.py:15-51; schemas implied by the call sites in
 *     quant_lstm.py:92-101 and modeling_rnnt.py:202-365), through the Python mirror
 *     rnnt_amd/ops.py.
 *
 * Plain pointers and sizes only.  Device pointers are HIP device allocations on the engine's
 * device; `stream` is a hipStream_t used as given (0 = the null stream).  Every entry point
 * returns 0 on success or a negative errno-style code; rnnt_last_error() describes the last
 * failure on the calling thread.  An engine is one batch in flight on one GPU, driven by one host
 * thread at a time; distinct engines (any number per GPU) are independent (the reference's per-socket
 * model clones, rnnt_model.hpp:45-46).  The C++ drop-in (csrc/sut/rnnt_model_mi355x.hpp) leases them
 * per call, so the reference SUT's threads never share one.
 */
#ifndef RNNT_MI355X_H
#define RNNT_MI355X_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RNNT_ABI_VERSION 8

#define RNNT_OK 0
#define RNNT_EINVAL (-22)
#define RNNT_ENOMEM (-12)
#define RNNT_EDEVICE (-5)

typedef struct rnnt_engine rnnt_engine;

/* Quantised / bf16 model in the reference's natural layouts (row = gate*H + unit, gate
 * order i,f,g,o).  Encoder layers l = 0..4 are pre_rnn.lstm0, lstm1, post_rnn.lstm0..2 with
 * input widths I = 256 (240 + zero pad), 1024, 2048, 1024, 1024 and K_l = I_l + 1024:
 * enc_w[l] = [W_ih_q | W_hh_q] int8 [4096][K_l]  (iLSTMLayer._quant_parameters, quant_lstm.py:193-215)
 * enc_bq[l] = (b_ih + b_hh) * s_in * s_w          fp32 [4096]
 * enc_rb / enc_in_s / enc_out_s                   the lstm_amx_int8 scale tensors (quant_lstm.py:92-101)
 * bf16 arrays hold bf16 bit patterns (torch .to(torch.bfloat16) of the checkpoint). */
typedef struct {
  const int8_t* enc_w[5];
  const float* enc_bq[5];
  float enc_rb[5], enc_in_s[5], enc_out_s[5];
  const uint16_t* embed;        /* bf16 [28][320] */
  const uint16_t* pred_w_ih[2]; /* bf16 [1280][320] */
  const uint16_t* pred_w_hh[2]; /* bf16 [1280][320] */
  const float* pred_b_ih[2];    /* fp32 [1280] */
  const float* pred_b_hh[2];    /* fp32 [1280] */
  const uint16_t* joint_w1t;    /* bf16 [512][1024]  joint.linear1_trans */
  const uint16_t* joint_w1p;    /* bf16 [512][320]   joint.linear1_pred */
  const float* joint_bt;        /* fp32 [512] */
  const float* joint_bp;        /* fp32 [512] */
  const uint16_t* joint_w2;     /* bf16 [29][512]    joint.linear2 */
  const float* joint_b2;        /* fp32 [29] */
} rnnt_model_desc;

typedef struct {
  int max_batch;   /* utterances per encode/decode call (default 1024) */
  int max_frames;  /* feature frames per utterance (default 500 = MAX_FEA_LEN, metadata.hpp:32) */
  int max_res;     /* result row length (default max_frames/2*30 = 7500, metadata.hpp:58-59) */
} rnnt_opts;

int rnnt_abi_version(void);
const char* rnnt_last_error(void);

/* Diagnostics, no reference counterpart: on SIGSEGV / SIGBUS / SIGFPE / SIGILL / SIGABRT print each
 * stack frame as shared object + offset to stderr, then pass the signal to the previously installed
 * handler.  bench.py installs it first thing. */
int rnnt_install_crash_report(void);

/* A HIP stream whose kernels run only on the CUs set in cu_mask (mask_words 32-bit words;
 * bit b = CU slot b/8 of XCD b%8 on MI355X; every XCD needs at least one bit), or a plain
 * non-blocking stream when cu_mask is NULL.  bench.py / the SUT keep the encoder off a few CUs
 * per XCD so the latency-bound greedy decode of the previous batch always finds free CUs.
 * Not a reference interface (the reference pins OpenMP teams to cores, torch_sut.cpp:143-149). */
int rnnt_stream_create(int device, const uint32_t* cu_mask, int mask_words, void** out);
int rnnt_stream_destroy(void* stream);

/* Packs the model into the engine's device layouts on `device` and sizes the workspace.
 * model == NULL gives an engine without weights: its components are loaded with the
 * rnnt_engine_load_* calls below (the operator library does this from the tensors the
 * TorchScript graph passes); a compute call whose component is missing fails with RNNT_EINVAL. */
int rnnt_engine_create(const rnnt_model_desc* model, int device, const rnnt_opts* opts, rnnt_engine** out);
void rnnt_engine_destroy(rnnt_engine* e);

/* The packed model file written by tools/export_model.py (rnnt_amd.weights.save_engine_file):
 * the rnnt_model_desc arrays in a flat little-endian container -- magic "RNNTMI01", u32 version 1,
 * u32 entry count, then per entry {char name[48]; u32 dtype (0 int8, 1 fp32, 2 bf16 bits);
 * u32 ndim; u64 shape[4]; u64 offset; u64 nbytes}, data 64-byte aligned.  Replaces the
 * reference's torch::jit::load of the calibrated TorchScript model (csrc/rnnt_model.hpp:41-54). */
int rnnt_engine_create_from_file(const char* path, int device, const rnnt_opts* opts, rnnt_engine** out);

/* Component loaders (natural layouts as in rnnt_model_desc); a reload overwrites the component in
 * place after synchronising the device.  Encoder layers [first, first + count): w[i], bq[i],
 * rb[i], in_s[i], out_s[i] for layer first + i (iLSTM.weights / rb_scale / in_scale / out_scale,
 * quant_lstm.py:92-101).  Prediction: embed may be NULL (operator-level use; the fused decode
 * needs it).  Joint: linear1 (w1t, w1p, bt, bp) and linear2 (w2 [29][512], b2 [29]). */
int rnnt_engine_load_encoder_layers(rnnt_engine* e, int first, int count, const int8_t* const* w,
                                    const float* const* bq, const float* rb, const float* in_s, const float* out_s);
int rnnt_engine_load_prediction(rnnt_engine* e, const uint16_t* embed, const uint16_t* const* w_ih,
                                const uint16_t* const* w_hh, const float* const* b_ih, const float* const* b_hh);
int rnnt_engine_load_joint(rnnt_engine* e, const uint16_t* w1t, const uint16_t* w1p, const float* bt, const float* bp);
int rnnt_engine_load_joint_out(rnnt_engine* e, const uint16_t* w2, const float* b2);

/* Encoder: feats device fp32 [T][n_pad][256] (the QSL's AssembleSamples layout, rnnt_qsl.cpp:150-188,
 * zero past lens and in channels 240..255), lens device int32 [n_pad] (0 for batch padding), lens_host
 * the same lengths on the host (drive the active-tile schedule; may be NULL = all T frames).
 * Keeps the encoder output (f, f_lens = ceil(lens/2)) in the engine for rnnt_engine_decode; if
 * f_out != NULL also writes f there, device fp32 [ceil(T/2)][n_pad][1024].
 * n_pad must be >= n, a multiple of 256, <= max_batch rounded up to 256. */
int rnnt_engine_encode(rnnt_engine* e, const float* feats, const int32_t* lens, const int32_t* lens_host,
                       int T, int n, int n_pad, float* f_out, void* stream);

/* encode with AssembleSamples (rnnt_qsl.cpp:150-188) fused into the input quantizer: the batch is
 * gathered straight from the QSL's ragged sample store -- store device fp32 [rows][240] (each
 * sample's [T_i][240] frames back to back, LoadSamplesToRam), offsets device int64 [n] (first
 * row of batch row i's sample), lens device int32 [n_pad] / lens_host int32 [n] (required; every
 * length <= T).  No assembled [T][n_pad][256] copy is made. */
int rnnt_engine_encode_gather(rnnt_engine* e, const float* store, const int64_t* offsets, const int32_t* lens,
                              const int32_t* lens_host, int T, int n, int n_pad, float* f_out, void* stream);

/* Greedy decode of the last encoded batch: res device int32 [n][max_res] (filled with -1 first),
 * res_len device int32 [n]. */
int rnnt_engine_decode(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res, void* stream);

/* ---- Server continuous batching (PipelineState, csrc/metadata.cpp:97-194; TorchModel::encode's
 * split_len loop, rnnt_model.hpp:62-90): the engine's rows are slots that carry their LSTM and
 * greedy state from one call to the next, so an utterance can be fed in chunks while finished
 * slots are refilled with new samples.
 * rnnt_engine_encode_stream: one chunk, gathered like rnnt_engine_encode_gather (offsets[i] = the
 * first stored frame of slot i's chunk, lens = the chunk's frames per slot, 0 for an idle slot).
 * reset device int32 [n_pad]: 1 = a new utterance starts in this slot (its h/c start at zero, the
 * masked_fill_ of PipelineState::update), 0 = continue from the slot's state after the previous
 * chunk.  Every chunk of an utterance but its last must have an even length (StackTime pairs
 * frames within the chunk).  n_pad is fixed for an engine's stream (the slot count).
 * rnnt_engine_decode_stream: greedy decode of that chunk's frames (f_lens = ceil(lens/2)) carrying
 * pre_g / pre_hg / pre_cg and the result row: a slot flagged in reset starts from SOS with
 * res[i] = -1 and res_len[i] = 0; the others append to res[i] (same buffer every call, max_res
 * the full utterance's bound).  res_len[i] = the slot's total symbols so far. */
int rnnt_engine_encode_stream(rnnt_engine* e, const float* store, const int64_t* offsets, const int32_t* lens,
                              const int32_t* lens_host, const int32_t* reset, int T, int n, int n_pad, void* stream);
int rnnt_engine_decode_stream(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res, const int32_t* reset,
                              void* stream);
/* Pipelined form of the two calls above: chunk k+1's rnnt_engine_encode_stream_pl may run (on its
 * own stream, from its own host thread) while chunk k's rnnt_engine_decode_stream_pl runs on
 * another.  Chunk k's encode copies its output to the decode side once chunk k-1's decode has read
 * it (encode_stream_pl blocks on the host until that decode has started); decode_stream_pl k must
 * be called after encode_stream_pl k returned, decodes in chunk order from one thread, encodes in
 * chunk order from one thread.  Chunk k's reset flags (read by its encode and its decode) must
 * stay unchanged until its decode has completed on the device.  The first encode_stream_pl puts
 * the engine in pipelined mode for good: its work is ordered after the engine's earlier calls, and
 * from then on the other encode / decode / op calls on that engine return RNNT_EINVAL. */
int rnnt_engine_encode_stream_pl(rnnt_engine* e, const float* store, const int64_t* offsets, const int32_t* lens,
                                 const int32_t* lens_host, const int32_t* reset, int T, int n, int n_pad,
                                 void* stream);
int rnnt_engine_decode_stream_pl(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res, const int32_t* reset,
                                 void* stream);

/* encode + decode. */
int rnnt_engine_infer(rnnt_engine* e, const float* feats, const int32_t* lens, const int32_t* lens_host, int T,
                      int n, int n_pad, int32_t* res, int32_t* res_len, int max_res, void* stream);

/* ---- fp32 transcription (BASELINE config 2; the reference's run_mode="f32" encoder,
 * models/modeling_rnnt.py:116-144 with torch LSTM layers).  Weights in the checkpoint's natural
 * layouts: wih[l] fp32 [4096][I_l] (I = 240, 1024, 2048, 1024, 1024), whh[l] fp32 [4096][1024],
 * bih[l] / bhh[l] fp32 [4096] (gate order i,f,g,o).  Optional; loaded once per engine. */
int rnnt_engine_load_f32_encoder(rnnt_engine* e, const float* const* wih, const float* const* whh,
                                 const float* const* bih, const float* const* bhh);
/* feats device fp32 [T][n_pad][256] (channels 240..255 ignored), lens device int32 [n_pad];
 * f_out device fp32 [ceil(T/2)][n_pad][1024] or NULL.  n_pad a multiple of 64.  Arithmetic: k-ordered
 * fp32 fma chains (b_ih + x.W_ih^T, b_hh + h.W_hh^T) on v_mfma_f32_16x16x4_f32, exact vs the CPU
 * restatement (oracle_encoder_f32).  Keeps f for rnnt_engine_decode_f32 (the fp32 decoder) and, when
 * n_pad <= max_batch (rounded up to 256), a bf16 copy for rnnt_engine_decode: the reference's
 * run_mode="f32" + enable_bf16 path, which converts f to bf16 before the joint (decoder.py:121-122). */
int rnnt_engine_encode_f32(rnnt_engine* e, const float* feats, const int32_t* lens, int T, int n, int n_pad,
                           float* f_out, void* stream);

/* ---- fp32 decoder (the run_mode="f32" Prediction / Joint with P.lstm and fp32 Linear layers,
 * modeling_rnnt.py:183-205, 285-288, and GreedyDecoder.greedy_decode_f32, decoder.py:102-169).
 * Natural layouts, fp32: embed [28][320], pred_w_ih/w_hh [2][1280][320] (gate order i,f,g,o),
 * pred_b_ih/b_hh [2][1280], joint_w1t [512][1024], joint_w1p [512][320], joint_bt/bp [512]
 * (bt = 0 after migrate_state_dict, utils.py:69), joint_w2 [29][512], joint_b2 [29]. */
typedef struct {
  const float* embed;
  const float* pred_w_ih[2];
  const float* pred_w_hh[2];
  const float* pred_b_ih[2];
  const float* pred_b_hh[2];
  const float* joint_w1t;
  const float* joint_w1p;
  const float* joint_bt;
  const float* joint_bp;
  const float* joint_w2;
  const float* joint_b2;
} rnnt_f32_decoder_desc;
int rnnt_engine_load_f32_decoder(rnnt_engine* e, const rnnt_f32_decoder_desc* d);
/* Greedy decode of the last rnnt_engine_encode_f32 output in fp32 (k-ordered fp32 fma chains on
 * v_mfma_f32_16x16x4_f32, exact vs oracle_greedy_decode with bf16 = 0); res / res_len as
 * rnnt_engine_decode. */
int rnnt_engine_decode_f32(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res, void* stream);

/* ---- in-run measurement (bench.py's roofline leg): HIP events recorded on the launch stream
 * around each call's encoder kernels and decoder kernels; rnnt_engine_get_stats synchronises
 * on the recorded events and sums their elapsed times. */
typedef struct {
  double encode_ms;       /* first to last encoder kernel of each encode call (step kernels + gaps) */
  double joint_trans_ms;  /* the F = b_t + f.W1t^T GEMM */
  double greedy_ms;       /* the device-side greedy decode loop */
  int64_t step_launches;  /* encoder tick kernels launched */
  int64_t decode_steps;   /* greedy lock-step iterations enqueued */
  int64_t encode_calls, decode_calls;
} rnnt_stats;
int rnnt_engine_set_profiling(rnnt_engine* e, int on);
/* Tick tile shape of the int8 encoder: "auto" (per tick, the cost model; the default), or pinned
 * to "big" (256 x 256), "small" (128 x 128, 2-deep ring), "tiny" (128 x 128, 4-deep) or "mini"
 * (64 x 128, 4-deep) -- results are identical (int32 accumulation); for tests and sweeps.  "flow":
 * whole-call encodes of batches with n_pad <= 256 run as one persistent dataflow launch (opt-in:
 * measured slower than the ticks on config 3); "ticks" = "auto".  The
 * environment variable RNNT_ENC_TILE sets an engine's initial value at create (development builds only). */
int rnnt_engine_set_tile(rnnt_engine* e, const char* tile);
/* Greedy decode tail: once at most `rows` rows of a decode call are still live, one persistent
 * launch runs every remaining lock-step step (weight slices kept in registers, phases handed off
 * through device counters; results identical) instead of four launches per step.  0 = off,
 * 1..512; in development builds the environment variable RNNT_DEC_PERSIST_ROWS sets an engine's
 * initial value.  The launch needs its 48 + (joint row groups, <= 32) workgroups resident at once:
 * beside other kernels a wait can time out, and rnnt_engine_decode then fails (RNNT_EDEVICE,
 * "persistent decode timed out").  No reference counterpart (the reference's loop is
 * rnnt_model.hpp:92-124). */
int rnnt_engine_set_decode_persist(rnnt_engine* e, int rows);
int rnnt_engine_get_stats(rnnt_engine* e, rnnt_stats* out, int reset);

/* ---- operator-level entry points (torch.ops.intel_mlperf mirror, rnnt_amd/ops.py) ---- */

/* lstm_amx_int8 for the engine's encoder layers [first, first+count): x = layer `first` input
 * (fp32 [T][n_pad][256] when first == 0, quantised in-kernel with in_s[0]; else int8
 * [T][n_pad][I_first]); hx int8 [count][n_pad][1024] and cx fp16 [count][n_pad][1024] in/out;
 * y: int8 [T][n_pad][1024], or fp32 when the last layer is the encoder's final layer (skip_quant_y).
 * Stacking between layers 1 and 2 is NOT applied here (callers use rnnt_op_stack_time). */
int rnnt_op_lstm_int8(rnnt_engine* e, int first, int count, const void* x, int T, int n_pad, int8_t* hx,
                      uint16_t* cx, void* y, void* stream);

/* stack_time(x int8 [T][n_pad][C], x_lens int32 [n_pad], factor 2) -> y int8 [ceil(T/2)][n_pad][2C]
 * (modeling_rnnt.py:326-328). */
int rnnt_op_stack_time(rnnt_engine* e, const int8_t* x, const int32_t* x_lens, int T, int n_pad, int C,
                       int8_t* y, void* stream);

/* ---- operator-level decode (the reference's op-by-op loop, models/decoder.py:171-212, on the
 * bound model; same arithmetic as the fused rnnt_engine_decode).  Row counts n_pad are multiples
 * of 16; bf16 tensors hold bf16 bit patterns. */
/* lstm_amx_bf16 (modeling_rnnt.py:202): x bf16 [n_pad][320] (embedding rows, zero for SOS),
 * hx bf16 [2][n_pad][320], cx fp32 [2][n_pad][320] -> hy, cy (same shapes, must not alias the
 * inputs); g = hy[1]. */
int rnnt_op_lstm_bf16(rnnt_engine* e, const uint16_t* x, const uint16_t* hx, const float* cx, uint16_t* hy, float* cy,
                      int n_pad, void* stream);
/* amx_linear_bf16_accum_relu (modeling_rnnt.py:269-275): f fp32 [n_pad][1024] (rounded to bf16),
 * g bf16 [n_pad][320] -> y1 bf16 [n_pad][512] = relu(f.W1t^T + b_t + g.W1p^T + b_p). */
int rnnt_op_joint_hidden(rnnt_engine* e, const float* f, const uint16_t* g, uint16_t* y1, int n_pad, void* stream);
/* amx_linear_i16o32 (modeling_rnnt.py:280-283): y1 bf16 [n_pad][512] -> logits fp32 [n_pad][32]
 * (labels 29..31 are zero padding, as the reference's padded linear2). */
int rnnt_op_joint_logits(rnnt_engine* e, const uint16_t* y1, float* logits, int n_pad, void* stream);
/* greedy_decode_update (modeling_rnnt.py:331-365; spec decoder.py:125-167), in place, on the
 * reference's own operands (the C++ decode loop's tensors, rnnt_model.hpp:92-124): symbols [n]
 * (int64 from torch.argmax when symbols_i64, else int32), symbols_added / res_idx / time_idx /
 * pre_g int32 [n], res int32 [n][max_res], f fp32 [Tp][f_batch][1024], f_lens int32 [n], fi fp32
 * [n][1024], pre_hg[l] / hg[l] bf16 [n][320], pre_cg[l] / cg[l] fp32 [n][320] (l = 0, 1).  The
 * spec's per-row `finish` (decoder.py:106) is carried in time_idx: a row is finished once
 * time_idx >= f_lens (left unclamped when it finishes; fi is gathered at min(time, f_len - 1)).
 * Synchronises the stream; returns 1 when every row has finished (the op's bool), 0 otherwise, or
 * a negative error code. */
int rnnt_op_greedy_update(rnnt_engine* e, const void* symbols, int symbols_i64, int32_t* symbols_added, int32_t* res,
                          int32_t* res_idx, const float* f, int f_batch, const int32_t* f_lens, int32_t* time_idx,
                          float* fi, int32_t* pre_g, uint16_t* const* pre_hg, float* const* pre_cg,
                          const uint16_t* const* hg, const float* const* cg, int n, int max_res, void* stream);

/* ---- operator-level fp32 prediction LSTM (intel_mlperf::lstm, modeling_rnnt.py:204, the
 * run_mode="f32" decoder): weights natural fp32 [1280][320] per layer (torch.nn.LSTM gate order
 * i, f, g, o), b_ih / b_hh [1280].  The same k-ordered fp32 chains as rnnt_engine_decode_f32. */
int rnnt_engine_load_f32_prediction(rnnt_engine* e, const float* const* w_ih, const float* const* w_hh,
                                    const float* const* b_ih, const float* const* b_hh);
/* x fp32 [n_pad][320] (embedding rows, zero for SOS), hx / cx fp32 [2][n_pad][320] -> hy, cy (same
 * shapes, must not alias the inputs); g = hy[1].  n_pad a multiple of 64. */
int rnnt_op_lstm_f32(rnnt_engine* e, const float* x, const float* hx, const float* cx, float* hy, float* cy,
                     int n_pad, void* stream);

/* ---- the audio processor's plugin operators one at a time (features.py:196-250; the graph
 * processor_jit.pt binds to; the fused rnnt_featurizer_run below is the throughput path).  No
 * engine needed; all device pointers, fp32 unless stated. */
/* preemphasis(x, x_lens, coeff, pad_size): row n (len lens[n] <= stride, at x + n * stride) ->
 * y [n][L_out]: y[p] = z[mirror(p - pad)] for p < len + 2 pad, z[0] = x[0], z[t] = x[t] - coeff
 * x[t-1] (torch reflect padding, periodic for short rows), 0 past it. */
int rnnt_op_preemphasis(const float* x, int64_t stride, const int32_t* lens, int n, int L_out, float coeff, int pad,
                        float* y, void* stream);
/* power_spectrum(x, x_lens): x [n][T][bins][2] (re, im) -> y [n][T][bins] = re^2 + im^2 for frames
 * t < frames[n], 0 after. */
int rnnt_op_power_spectrum(const float* x, const int32_t* frames, int n, int T, int bins, float* y, void* stream);
/* frame_splicing(x, x_lens, factor): x [n][C][T] -> y [n][C factor][ceil(T / factor)],
 * y[q C + m][t] = x[m][factor t + q] for stacked frames < frames[n], 0 otherwise. */
int rnnt_op_frame_splicing(const float* x, const int32_t* frames, int n, int C, int T, int factor, float* y,
                           void* stream);
/* i_layernorm_pad(x, weight, bias, x_lens, eps, unbiased, output_shape): x [n][C][T], weight / bias
 * [C_out][wt] -> y [n_out][C_out][T]: per row and channel over its lens[n] valid frames,
 * (x - mean) / sqrt(var + eps) * weight + bias (var unbiased when asked; 0 for one frame), zero past
 * the length, in channels >= C and rows >= n; lens_out int32 [n_out]. */
int rnnt_op_layernorm_pad(const float* x, const float* weight, const float* bias, int wt, const int32_t* lens, int n,
                          int C, int T, int n_out, int C_out, float eps, int unbiased, float* y, int32_t* lens_out,
                          void* stream);

/* ---- audio front end (the reference's AudioProcessor / FilterbankFeatures.forward,
 * datasets/parts/features.py:185-252, csrc/rnnt_processor.hpp:29-48; used when WAV=true,
 * launch_sut.sh:54).  Geometry fixed to configs/rnnt.toml [input_eval]; the window and filterbank
 * are the module's buffers (torch.hann_window(320, periodic=False), librosa.filters.mel(16000, 512,
 * 80) -- features.py:134-154), passed in as data. */
typedef struct rnnt_featurizer rnnt_featurizer;
typedef struct {
  int sample_rate;     /* 16000 */
  int n_fft;           /* 512 */
  int win_length;      /* 320 = sample_rate * window_size */
  int hop_length;      /* 160 = sample_rate * window_stride */
  int nfilt;           /* 80 */
  int frame_splicing;  /* 3 */
  int pad_out_feat;    /* 256 (run_mode quant: pad_out_feat=True, process_librispeech.py:104) */
  float preemph;       /* 0.97 (0 disables) */
  float dither;        /* 1e-5: dither^2 is added to the power spectrum (features.py:219-220) */
  float log_guard;     /* fb_bias 1e-20 (features.py:158-160) */
  float norm_eps;      /* i_layernorm_pad eps 1e-12 (features.py:243-249) */
} rnnt_featurizer_config;

/* window host fp32 [win_length]; fb host fp32 [nfilt][n_fft/2+1]. */
int rnnt_featurizer_create(const rnnt_featurizer_config* cfg, const float* window, const float* fb, int device,
                           rnnt_featurizer** out);
void rnnt_featurizer_destroy(rnnt_featurizer* f);
/* The same from the processor file tools/export_model.py --processor-file writes (the RNNTMI01
 * container: fz_config fp32 [11] = the config fields in order, fz_window fp32 [win_length], fz_fb fp32
 * [nfilt][n_fft/2+1]); replaces torch::jit::load of the TorchScript processor (rnnt_processor.hpp:17-22). */
int rnnt_featurizer_create_from_file(const char* path, int device, rnnt_featurizer** out);
/* Dynamic LDS each fz_logmel workgroup requests so that it owns its CU (environment RNNT_FZ_OWN_CU=1 at
 * create; 0 = off, the default).  A fallback guard beside the shipped one (no packed FP32 in any
 * kernel); no reference counterpart. */
size_t rnnt_featurizer_own_cu_lds(const rnnt_featurizer* f);
/* Feature frames of a wav_len-sample utterance: ceil((1 + floor(wav_len/hop)) / 3), 0 for 0. */
int64_t rnnt_featurizer_frames(int64_t wav_len);
/* wav device fp32: row n's samples at wav + offsets[n] (offsets device int64 [n]) or, with
 * offsets == NULL, at wav + n * stride (the reference's zero-padded [N][maxLength] batch,
 * rnnt_qsl.cpp:166-179).  wav_lens device int32 [n] and the same on the host (wav_lens_host).
 * Writes feats device fp32 [T_out][n_pad][256] -- the encoder's input layout -- normalised per
 * utterance and channel, zero past feat_lens[n], in channels 240..255 and in rows n..n_pad-1;
 * feat_lens device int32 [n_pad].  T_out >= the longest utterance's frames (else RNNT_EINVAL).
 * The reference returns [n_pad][256][T] (features.py:241-250); the C++ SUT permutes it to this
 * layout before encode (torch_sut.cpp:200). */
int rnnt_featurizer_run(rnnt_featurizer* f, const float* wav, const int64_t* offsets, int64_t stride,
                        const int32_t* wav_lens, const int32_t* wav_lens_host, int n, int n_pad, float* feats,
                        int32_t* feat_lens, int T_out, void* stream);
/* Ragged variant for a feature store (the Server producer: featurize arriving samples once, the
 * consumer encodes from the store, rnnt_engine_encode_stream): the same features, frame t of row
 * n written as 240 fp32 at feats + (row_off[n] + t) * 240 (row_off device int64 [n]), nothing
 * else touched; feat_lens device int32 [n].  Every row's frames <= max_frames (else RNNT_EINVAL). */
int rnnt_featurizer_run_rows(rnnt_featurizer* f, const float* wav, const int64_t* offsets, int64_t stride,
                             const int32_t* wav_lens, const int32_t* wav_lens_host, int n, float* feats,
                             const int64_t* row_off, int32_t* feat_lens, int max_frames, void* stream);

#ifdef __cplusplus
}
#endif
#endif

// engine.hip -- C ABI of the MI355X RNN-T engine (include/rnnt_mi355x.h).
//
// Host side: model packing into device layouts, workspace management and the per-batch
// launch schedule (the replacement of TorchModel::encode / decode, reference
// csrc/rnnt_model.hpp:62-124).  No torch types anywhere: plain pointers and sizes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rnnt_mi355x.h"
#include "decoder.hpp"
#include "decoder_ops.hpp"
#include "encoder.hpp"
#include <hip/hip_ext.h>
#include "encoder_f32.hpp"
#include "decoder_f32.hpp"
#include "rnnt_device.hpp"

using namespace rnnt;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int rnnt_internal_fail(int code, const std::string& msg) { return fail(code, msg); }
#define DEVICE_SCOPE(dev)                                                                      \
  DeviceScope dscope_(dev);                                                                    \
  if (!dscope_.ok) return fail(RNNT_EDEVICE, "hipSetDevice failed")
#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return fail(RNNT_EDEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static const int ENC_I[5] = {256, 1024, 2048, 1024, 1024};

struct rnnt_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  rnnt_opts opts{};
  int np_max = 0, tp_max = 0;
  int tile = ENC_TILE_AUTO;  // tick tile shape / flow (rnnt_engine_set_tile; RNNT_ENC_TILE at create)
  int persist_rows = 0;      // persistent tail decode threshold (rnnt_engine_set_decode_persist; RNNT_DEC_PERSIST_ROWS at create)
  bool stream_prefix = false;  // stream chunks skip only trailing done tiles (RNNT_STREAM_PREFIX=1: A/B)
  // packed weights
  int8_t* enc_w[5] = {};
  float* enc_bq[5] = {};
  float rb[5], in_s[5], out_s[5];
  DecWeights dw{};
  std::vector<void*> allocs;
  // workspace
  int8_t *x0q = nullptr, *yA = nullptr, *xs = nullptr, *yB = nullptr, *yC = nullptr;
  int8_t* h[5][2] = {};
  uint16_t* c[5] = {};
  uint16_t* fbf = nullptr;
  float *F = nullptr, *hc = nullptr, *G = nullptr, *PH = nullptr;
  int32_t* flen = nullptr;
  DecState ds{};
  int32_t* host_flags = nullptr;
  hipEvent_t poll_ev[2] = {nullptr, nullptr};
  // last encoded batch
  int last_T = 0, last_n = 0, last_npad = 0;
  // h ping-pong: layer l's state before its step t sits in h[l][(t + hpar[l]) & 1]; a stream
  // (carried-state) encode advances hpar by the steps it ran
  int hpar[5] = {};
  // Stream ordering of the engine's own state (h/c, x0q, the encoder output, decode state):
  // every call that touches it waits for the previous such call's completion event, on
  // whatever stream that one ran, and records its own -- so encode -> decode -> next encode
  // are ordered even when the caller puts them on different streams.
  hipEvent_t state_ev = nullptr;
  bool state_rec = false;
  // Pipelined stream calls (rnnt_engine_encode_stream_pl / decode_stream_pl): chunk k+1's encode
  // runs while chunk k decodes.  The encoder keeps its own state in stream order; at the end of
  // chunk k's encode its final-layer output and lengths are copied to the decode side (fbf_dec,
  // flen_dec) once chunk k-1's decode has handed them off (after its joint_trans and its private
  // copy of the lengths).  Encode k waits for hand-off k-1 on the host (the condition below) and
  // on the GPU (pl_handoff_ev); decode k waits for copy k (pl_copy_ev[k & 1]).
  uint16_t* fbf_dec = nullptr;
  int32_t *flen_dec = nullptr, *flen_dpriv = nullptr;
  hipEvent_t pl_copy_ev[2] = {nullptr, nullptr}, pl_handoff_ev = nullptr;
  int pl_meta[2][3] = {};  // (T, n, n_pad) of chunk k at k & 1
  int64_t pl_enc_k = 0, pl_dec_k = 0, pl_handoff_k = -1;
  bool pl_failed = false;  // sticky: a pipelined decode failed; the encode side returns an error instead of waiting
  std::atomic<bool> pl_mode{false};  // set by the first pipelined call: the other calls then fail
  std::mutex pl_mu;
  std::condition_variable pl_cv;
  // profiling
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_enc;
  std::vector<std::array<hipEvent_t, 3>> ev_dec;
  int64_t step_launches = 0, decode_steps = 0, encode_calls = 0, decode_calls = 0;
  // optional fp32 encoder (rnnt_engine_load_f32_encoder) and its lazily sized workspace
  bool f32_loaded = false;
  float *f32_wih[5] = {}, *f32_whh[5] = {}, *f32_bih[5] = {}, *f32_bhh[5] = {};
  std::vector<void*> f32_ws;
  size_t f32_ws_T = 0, f32_ws_np = 0;
  float *f32_x = nullptr, *f32_ya = nullptr, *f32_xs = nullptr, *f32_yb = nullptr, *f32_yc = nullptr;
  float *f32_h[5][2] = {}, *f32_c[5] = {};  // per layer: the wavefront ticks run the layers concurrently
  // fp32 decoder (rnnt_engine_load_f32_decoder) and the last fp32 encode's outputs it decodes
  bool f32_dec_loaded = false, f32_pred_loaded = false;
  DecF32Weights dw32{};
  float *f32_fc = nullptr, *f32_F = nullptr;
  int32_t* f32_flen = nullptr;
  DecF32State ds32{};
  int last32_T = 0, last32_n = 0, last32_npad = 0;
  // persistent dataflow encoder (small batches, lstm_i8_flow_kernel): step table + task blocks on
  // the device (flow_dev), staged through pinned host memory (flow_host; flow_up_ev: the last
  // upload has consumed it), per-step counters (flow_ctr) and the last launch's abort word read
  // back into flow_abort (flow_done_ev)
  char *flow_dev = nullptr, *flow_host = nullptr;
  uint32_t* flow_ctr = nullptr;
  uint32_t* flow_abort = nullptr;
  size_t flow_cap = 0;  // steps
  hipEvent_t flow_up_ev = nullptr, flow_done_ev = nullptr;
  bool flow_up_pending = false, flow_check = false;
  int64_t flow_launches = 0;
  // operator-level decode: unfinished-row counter for greedy_decode_update's return value
  int32_t* op_count = nullptr;
  int32_t* op_count_host = nullptr;
  // which model components are on the device (rnnt_engine_create with a model loads all)
  int enc_loaded = 0;  // bit l: encoder layer l
  bool pred_loaded = false, xtab_ok = false, joint1_loaded = false, joint2_loaded = false;
};

static hipEvent_t new_event(hipStream_t st) {
  hipEvent_t ev = nullptr;
  if (hipEventCreate(&ev) == hipSuccess) (void)hipEventRecord(ev, st);
  return ev;
}

template <class T>
static int dev_alloc(rnnt_engine* e, T** p, size_t count) {
  void* q = nullptr;
  if (hipMalloc(&q, count * sizeof(T) + 256) != hipSuccess) return fail(RNNT_ENOMEM, "hipMalloc failed");
  e->allocs.push_back(q);
  *p = (T*)q;
  return 0;
}
template <class T>
static int upload(rnnt_engine* e, T** p, const std::vector<T>& host) {
  int r = dev_alloc(e, p, host.size());
  if (r) return r;
  HIPCHK(hipMemcpy(*p, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

extern "C" int rnnt_abi_version(void) { return RNNT_ABI_VERSION; }
extern "C" const char* rnnt_last_error(void) { return g_err.c_str(); }

// CU-partitioned streams (MI355X scheduling, not a reference interface): bit b of the mask is
// CU slot b/8 of XCD b%8 (probe: tools/probe/probe_cumask.hip); every XCD must keep >= 1 bit
// (an XCD with none is given all of its CUs by the runtime).
extern "C" int rnnt_stream_create(int device, const uint32_t* cu_mask, int mask_words, void** out) {
  if (!out || (cu_mask && (mask_words <= 0 || mask_words > 16))) return fail(RNNT_EINVAL, "rnnt_stream_create: bad mask");
  DEVICE_SCOPE(device);
  hipStream_t s = nullptr;
  if (cu_mask) {
    uint32_t per_xcd[8] = {0};
    for (int b = 0; b < 32 * mask_words; ++b)
      if (cu_mask[b >> 5] >> (b & 31) & 1u) per_xcd[b & 7]++;
    for (int x = 0; x < 8; ++x)
      if (!per_xcd[x]) return fail(RNNT_EINVAL, "rnnt_stream_create: every XCD needs at least one CU");
    HIPCHK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, cu_mask));
  } else {
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  *out = (void*)s;
  return RNNT_OK;
}
extern "C" int rnnt_stream_destroy(void* stream) {
  HIPCHK(hipStreamDestroy((hipStream_t)stream));
  return RNNT_OK;
}

// ---- packing (natural layouts -> device layouts; see DESIGN.md "Data layout in HBM").
// Each model component has a fixed-size device buffer, allocated on its first load and
// overwritten in place by a reload (the operator library reloads a component when the weight
// tensors it is called with change; the device is synchronised first so no kernel still reads
// the old copy).
template <class T>
static int load_buf(rnnt_engine* e, T** p, const std::vector<T>& host) {
  if (!*p) return upload(e, p, host);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(*p, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

extern "C" int rnnt_engine_load_encoder_layers(rnnt_engine* e, int first, int count, const int8_t* const* w,
                                               const float* const* bq, const float* rb, const float* in_s,
                                               const float* out_s) {
  if (!e || !w || !bq || !rb || !in_s || !out_s) return fail(RNNT_EINVAL, "null argument");
  if (first < 0 || count <= 0 || first + count > 5) return fail(RNNT_EINVAL, "bad encoder layer range");
  DEVICE_SCOPE(e->device);
  for (int i = 0; i < count; ++i) {
    const int l = first + i;
    if (!w[i] || !bq[i]) return fail(RNNT_EINVAL, "null encoder weight");
    const int K = ENC_I[l] + H;
    std::vector<int8_t> wp((size_t)G4 * K);
    std::vector<float> b(G4);
    for (int g = 0; g < 4; ++g)
      for (int u = 0; u < H; ++u) {
        const int pr = enc_packed_row(u, g);
        memcpy(&wp[(size_t)pr * K], w[i] + (size_t)(g * H + u) * K, K);
        // the cell's folded bias term, as oracle_enc_bias: (bq rb) * (g == 2 ? 128 : 64) + 1024
        const float bqr = bq[i][g * H + u] * rb[i];
        b[pr] = g == 2 ? bqr * 128.0f + 1024.0f : bqr * 64.0f + 1024.0f;
      }
    int r = load_buf(e, &e->enc_w[l], wp);
    if (!r) r = load_buf(e, &e->enc_bq[l], b);
    if (r) return r;
    e->rb[l] = rb[i];
    e->in_s[l] = in_s[i];
    e->out_s[l] = out_s[i];
    e->enc_loaded |= 1 << l;
  }
  return 0;
}

// prediction LSTM: rows gate-interleaved, k = [W_ih | W_hh] natural, biases separate (the two
// chains b_ih + x.W_ih and b_hh + h.W_hh are summed after, oracle pred_row).  embed may be NULL
// (operator-level use: the caller embeds); the fused decode needs it for its layer-0 table.
extern "C" int rnnt_engine_load_prediction(rnnt_engine* e, const uint16_t* embed, const uint16_t* const* w_ih,
                                           const uint16_t* const* w_hh, const float* const* b_ih,
                                           const float* const* b_hh) {
  if (!e || !w_ih || !w_hh || !b_ih || !b_hh) return fail(RNNT_EINVAL, "null argument");
  DEVICE_SCOPE(e->device);
  for (int l = 0; l < 2; ++l) {
    if (!w_ih[l] || !w_hh[l] || !b_ih[l] || !b_hh[l]) return fail(RNNT_EINVAL, "null prediction weight");
    std::vector<uint16_t> w((size_t)PG4 * 640);
    std::vector<float> b(2 * PG4);
    for (int g = 0; g < 4; ++g)
      for (int u = 0; u < P; ++u) {
        const int src = g * P + u, dst = 4 * u + g;
        for (int k = 0; k < 640; ++k)
          w[(size_t)dst * 640 + k] = k < P ? w_ih[l][(size_t)src * P + k] : w_hh[l][(size_t)src * P + k - P];
        b[dst] = b_ih[l][src];
        b[PG4 + dst] = b_hh[l][src];
      }
    uint16_t* dwp = const_cast<uint16_t*>(e->dw.wp[l]);
    float* dbp = const_cast<float*>(e->dw.bih_p[l]);
    int r = load_buf(e, &dwp, w);
    if (!r) r = load_buf(e, &dbp, b);
    if (r) return r;
    e->dw.wp[l] = dwp;
    e->dw.bih_p[l] = dbp;
    e->dw.bhh_p[l] = dbp + PG4;
  }
  e->pred_loaded = true;
  e->xtab_ok = false;
  if (embed) {
    uint16_t* emb = const_cast<uint16_t*>(e->dw.embed);
    int r = load_buf(e, &emb, std::vector<uint16_t>(embed, embed + 28 * P));
    if (r) return r;
    e->dw.embed = emb;
    // layer-0 input table (b_ih + emb[g].W_ih^T per label, same MFMA chain as the step kernels)
    float* xtab = const_cast<float*>(e->dw.xtab);
    if (!xtab && (r = dev_alloc(e, &xtab, (size_t)29 * PG4))) return r;
    DecWeights w = e->dw;
    if (launch_dec_xtab(w, xtab, e->stream)) return fail(RNNT_EDEVICE, "xtab launch failed");
    HIPCHK(hipStreamSynchronize(e->stream));
    e->dw.xtab = xtab;
    e->xtab_ok = true;
  }
  return 0;
}

// joint first layer: linear1_trans (w1t [512][1024], bt) and linear1_pred (w1p [512][320], bp)
extern "C" int rnnt_engine_load_joint(rnnt_engine* e, const uint16_t* w1t, const uint16_t* w1p, const float* bt,
                                      const float* bp) {
  if (!e || !w1t || !w1p || !bt || !bp) return fail(RNNT_EINVAL, "null argument");
  DEVICE_SCOPE(e->device);
  uint16_t *dt = const_cast<uint16_t*>(e->dw.w1t), *dp = const_cast<uint16_t*>(e->dw.w1p);
  float *dbt = const_cast<float*>(e->dw.bt), *dbp = const_cast<float*>(e->dw.bp);
  int r = load_buf(e, &dt, std::vector<uint16_t>(w1t, w1t + (size_t)J * H));
  if (!r) r = load_buf(e, &dp, std::vector<uint16_t>(w1p, w1p + (size_t)J * P));
  if (!r) r = load_buf(e, &dbt, std::vector<float>(bt, bt + J));
  if (!r) r = load_buf(e, &dbp, std::vector<float>(bp, bp + J));
  if (r) return r;
  e->dw.w1t = dt; e->dw.w1p = dp; e->dw.bt = dbt; e->dw.bp = dbp;
  e->joint1_loaded = true;
  return 0;
}

// joint output layer: linear2 (w2 [29][512], b2 [29]), zero-padded to 32 labels
extern "C" int rnnt_engine_load_joint_out(rnnt_engine* e, const uint16_t* w2, const float* b2) {
  if (!e || !w2 || !b2) return fail(RNNT_EINVAL, "null argument");
  DEVICE_SCOPE(e->device);
  std::vector<uint16_t> w((size_t)NLAB_PAD * J, 0);
  std::copy(w2, w2 + (size_t)NLAB * J, w.begin());
  std::vector<float> b(NLAB_PAD, 0.0f);
  std::copy(b2, b2 + NLAB, b.begin());
  uint16_t* dw2 = const_cast<uint16_t*>(e->dw.w2);
  float* db2 = const_cast<float*>(e->dw.b2);
  int r = load_buf(e, &dw2, w);
  if (!r) r = load_buf(e, &db2, b);
  if (r) return r;
  e->dw.w2 = dw2;
  e->dw.b2 = db2;
  e->joint2_loaded = true;
  return 0;
}

static int pack_model(rnnt_engine* e, const rnnt_model_desc* m) {
  if (!m->embed || !m->joint_w1t || !m->joint_w1p || !m->joint_w2 || !m->joint_bt || !m->joint_bp || !m->joint_b2)
    return fail(RNNT_EINVAL, "null joint/embedding weight");
  int r = rnnt_engine_load_encoder_layers(e, 0, 5, m->enc_w, m->enc_bq, m->enc_rb, m->enc_in_s, m->enc_out_s);
  if (!r) r = rnnt_engine_load_prediction(e, m->embed, m->pred_w_ih, m->pred_w_hh, m->pred_b_ih, m->pred_b_hh);
  if (!r) r = rnnt_engine_load_joint(e, m->joint_w1t, m->joint_w1p, m->joint_bt, m->joint_bp);
  if (!r) r = rnnt_engine_load_joint_out(e, m->joint_w2, m->joint_b2);
  return r;
}

static int alloc_workspace(rnnt_engine* e) {
  const size_t NP = e->np_max, TM = e->opts.max_frames, TPM = e->tp_max;
  int r = 0;
  r = r ? r : dev_alloc(e, &e->x0q, TM * NP * FEAT);
  r = r ? r : dev_alloc(e, &e->yA, TM * NP * H);
  r = r ? r : dev_alloc(e, &e->xs, TPM * NP * 2 * H);
  r = r ? r : dev_alloc(e, &e->yB, TPM * NP * H);
  r = r ? r : dev_alloc(e, &e->yC, TPM * NP * H);
  for (int l = 0; l < 5 && !r; ++l) {
    r = r ? r : dev_alloc(e, &e->h[l][0], NP * H);
    r = r ? r : dev_alloc(e, &e->h[l][1], NP * H);
    r = r ? r : dev_alloc(e, &e->c[l], NP * H);
  }
  r = r ? r : dev_alloc(e, &e->fbf, TPM * NP * H);
  r = r ? r : dev_alloc(e, &e->F, TPM * NP * J);
  r = r ? r : dev_alloc(e, &e->hc, NP * 2 * 4 * P);
  r = r ? r : dev_alloc(e, &e->G, NP * J);
  r = r ? r : dev_alloc(e, &e->PH, NP * PG4);
  r = r ? r : dev_alloc(e, &e->flen, NP);
  int32_t** ints[] = {&e->ds.time, &e->ds.added, &e->ds.idx, &e->ds.preg, &e->ds.slot, &e->ds.fin};
  for (auto pp : ints) r = r ? r : dev_alloc(e, pp, NP);
  r = r ? r : dev_alloc(e, &e->ds.list, 2 * NP);
  r = r ? r : dev_alloc(e, &e->ds.live, 2 * NP);  // int4 entries
  r = r ? r : dev_alloc(e, &e->ds.count, 4);
  r = r ? r : dev_alloc(e, &e->ds.unfinished, 4);
  r = r ? r : dev_alloc(e, &e->ds.pc, 8);
  if (!r && hipHostMalloc((void**)&e->host_flags, 4 * sizeof(int32_t), hipHostMallocDefault) != hipSuccess)
    r = fail(RNNT_ENOMEM, "hipHostMalloc failed");
  for (int i = 0; i < 2 && !r; ++i)
    if (hipEventCreateWithFlags(&e->poll_ev[i], hipEventDisableTiming) != hipSuccess)
      r = fail(RNNT_EDEVICE, "hipEventCreate failed");
  if (!r && hipEventCreateWithFlags(&e->state_ev, hipEventDisableTiming) != hipSuccess)
    r = fail(RNNT_EDEVICE, "hipEventCreate failed");
  return r;
}

extern "C" void rnnt_engine_destroy(rnnt_engine* e) {
  if (!e) return;
  DeviceScope dscope(e->device);
  for (void* p : e->allocs) (void)hipFree(p);
  for (void* p : e->f32_ws) (void)hipFree(p);
  if (e->op_count_host) (void)hipHostFree(e->op_count_host);
  if (e->host_flags) (void)hipHostFree(e->host_flags);
  for (auto ev : {e->flow_up_ev, e->flow_done_ev})
    if (ev) {
      (void)hipEventSynchronize(ev);
      (void)hipEventDestroy(ev);
    }
  if (e->flow_host) (void)hipHostFree(e->flow_host);
  if (e->flow_abort) (void)hipHostFree(e->flow_abort);
  for (auto ev : e->poll_ev)
    if (ev) (void)hipEventDestroy(ev);
  for (auto ev : {e->pl_copy_ev[0], e->pl_copy_ev[1], e->pl_handoff_ev})
    if (ev) (void)hipEventDestroy(ev);
  if (e->state_ev) {
    (void)hipEventSynchronize(e->state_ev);
    (void)hipEventDestroy(e->state_ev);
  }
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

static int tile_code(const char* s) {
  if (!strcmp(s, "auto")) return ENC_TILE_AUTO;
  if (!strcmp(s, "big")) return ENC_TILE_BIG;
  if (!strcmp(s, "small")) return ENC_TILE_SMALL;
  if (!strcmp(s, "tiny")) return ENC_TILE_TINY;
  if (!strcmp(s, "mini")) return ENC_TILE_MINI;
  if (!strcmp(s, "flow")) return ENC_TILE_FLOW;
  if (!strcmp(s, "ticks")) return ENC_TILE_TICKS;
  return -1;
}

extern "C" int rnnt_engine_set_tile(rnnt_engine* e, const char* tile) {
  if (!e || !tile) return fail(RNNT_EINVAL, "null argument");
  const int v = tile_code(tile);
  if (v < 0) return fail(RNNT_EINVAL, std::string("unknown tick tile '") + tile + "': auto|ticks|flow|big|small|tiny|mini");
  e->tile = v;
  return 0;
}

extern "C" int rnnt_engine_set_decode_persist(rnnt_engine* e, int rows) {
  if (!e) return fail(RNNT_EINVAL, "null argument");
  if (rows < 0 || rows > DEC_PERSIST_MAX) return fail(RNNT_EINVAL, "persistent decode rows must be 0 (off) .. 512");
  e->persist_rows = rows;
  return 0;
}

extern "C" int rnnt_engine_create(const rnnt_model_desc* model, int device, const rnnt_opts* opts,
                                  rnnt_engine** out) {
  if (!out) return fail(RNNT_EINVAL, "null argument");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RNNT_EDEVICE, "no HIP device");
  if (device < 0 || device >= ndev) return fail(RNNT_EINVAL, "bad device index");
  rnnt_engine* e = new rnnt_engine();
  e->device = device;
  e->opts.max_batch = (opts && opts->max_batch > 0) ? opts->max_batch : 1024;
  e->opts.max_frames = (opts && opts->max_frames > 0) ? opts->max_frames : 500;
  e->opts.max_res = (opts && opts->max_res > 0) ? opts->max_res : (e->opts.max_frames / 2) * MAXSYM;
  e->np_max = (e->opts.max_batch + ENC_PAD - 1) / ENC_PAD * ENC_PAD;
  e->tp_max = (e->opts.max_frames + 1) / 2;
  int r = 0;
  // decode live-list entries hold the row in 24 bits and the frame / f_len in 16 bits each
  if (e->np_max >= (1 << 24) || e->tp_max > 0xffff) r = fail(RNNT_EINVAL, "max_batch or max_frames too large");
  DeviceScope dscope(device);
  if (!r && !dscope.ok) r = fail(RNNT_EDEVICE, "hipSetDevice failed");
  if (!r && hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
    r = fail(RNNT_EDEVICE, "hipStreamCreate failed");
  if (const char* pr = dev_env("RNNT_DEC_PERSIST_ROWS")) {  // development default, read once per engine
    const int v = atoi(pr);
    e->persist_rows = v < 0 ? 0 : (v > DEC_PERSIST_MAX ? DEC_PERSIST_MAX : v);
  }
  if (const char* t = dev_env("RNNT_ENC_TILE")) {  // development default, read once per engine
    const int v = tile_code(t);
    if (v < 0) r = fail(RNNT_EINVAL, std::string("RNNT_ENC_TILE=") + t + ": auto|ticks|flow|big|small|tiny|mini");
    e->tile = v < 0 ? ENC_TILE_AUTO : v;
  }
  {
    const char* sp = dev_env("RNNT_STREAM_PREFIX");
    e->stream_prefix = sp && atoi(sp) != 0;
  }
  if (!r && model) r = pack_model(e, model);
  if (!r) r = alloc_workspace(e);
  if (r) {
    rnnt_engine_destroy(e);
    return r;
  }
  *out = e;
  return 0;
}

// ---- packed model file (include/rnnt_mi355x.h: rnnt_engine_create_from_file)
namespace {
struct PkEntry {
  char name[48];
  uint32_t dtype, ndim;
  uint64_t shape[4];
  uint64_t offset, nbytes;
};
static_assert(sizeof(PkEntry) == 48 + 8 + 32 + 16, "packed entry layout");
}  // namespace

// the container read into memory, entries looked up by name with type / shape / extent checked
struct PackFile {
  std::vector<char> buf;
  std::vector<PkEntry> ents;
  std::string where;
  int load(const char* path) {
    FILE* fp = fopen(path, "rb");
    if (!fp) return fail(RNNT_EINVAL, std::string("cannot open ") + path);
    char tmp[1 << 16];
    size_t k;
    while ((k = fread(tmp, 1, sizeof(tmp), fp)) > 0) buf.insert(buf.end(), tmp, tmp + k);
    fclose(fp);
    where = std::string(path) + ": ";
    if (buf.size() < 16 || memcmp(buf.data(), "RNNTMI01", 8) != 0) return fail(RNNT_EINVAL, where + "not an RNNTMI01 file");
    uint32_t version = 0, count = 0;
    memcpy(&version, buf.data() + 8, 4);
    memcpy(&count, buf.data() + 12, 4);
    if (version != 1 || count > 256 || 16 + (size_t)count * sizeof(PkEntry) > buf.size())
      return fail(RNNT_EINVAL, where + "bad header");
    ents.resize(count);
    memcpy(ents.data(), buf.data() + 16, count * sizeof(PkEntry));
    return 0;
  }
  // name -> data (dtype 0 int8, 1 fp32, 2 bf16 bits; `elems` elements)
  int find(const std::string& name, uint32_t dtype, uint64_t elems, const void** ptr) const {
    for (const PkEntry& en : ents) {
      if (strncmp(en.name, name.c_str(), sizeof(en.name)) != 0) continue;
      uint64_t n = 1;
      for (uint32_t d = 0; d < en.ndim && d < 4; ++d) n *= en.shape[d];
      const uint64_t esz = dtype == 0 ? 1 : dtype == 1 ? 4 : 2;
      if (en.dtype != dtype || en.ndim > 4 || n != elems || en.nbytes != n * esz || en.offset % 64 ||
          en.offset > buf.size() || en.nbytes > buf.size() - en.offset)
        return fail(RNNT_EINVAL, where + "entry " + name + " has the wrong type, shape or extent");
      *ptr = buf.data() + en.offset;
      return 0;
    }
    return fail(RNNT_EINVAL, where + "missing entry " + name);
  }
};

extern "C" int rnnt_engine_create_from_file(const char* path, int device, const rnnt_opts* opts, rnnt_engine** out) {
  if (!path || !out) return fail(RNNT_EINVAL, "null argument");
  *out = nullptr;
  PackFile pf;
  if (int r0 = pf.load(path)) return r0;
  auto find = [&](const std::string& name, uint32_t dtype, uint64_t elems, const void** ptr) {
    return pf.find(name, dtype, elems, ptr);
  };
  rnnt_model_desc d{};
  int r = 0;
  const void* p = nullptr;
  const float* rb = nullptr;
  const float* ins = nullptr;
  const float* outs = nullptr;
  for (int l = 0; l < 5 && !r; ++l) {
    if (!(r = find("enc_w." + std::to_string(l), 0, (uint64_t)G4 * (ENC_I[l] + H), &p))) d.enc_w[l] = (const int8_t*)p;
    if (!r && !(r = find("enc_bq." + std::to_string(l), 1, G4, &p))) d.enc_bq[l] = (const float*)p;
  }
  if (!r && !(r = find("enc_rb", 1, 5, &p))) rb = (const float*)p;
  if (!r && !(r = find("enc_in_s", 1, 5, &p))) ins = (const float*)p;
  if (!r && !(r = find("enc_out_s", 1, 5, &p))) outs = (const float*)p;
  if (!r) {
    memcpy(d.enc_rb, rb, sizeof(d.enc_rb));
    memcpy(d.enc_in_s, ins, sizeof(d.enc_in_s));
    memcpy(d.enc_out_s, outs, sizeof(d.enc_out_s));
  }
  if (!r && !(r = find("embed", 2, (uint64_t)28 * P, &p))) d.embed = (const uint16_t*)p;
  for (int l = 0; l < 2 && !r; ++l) {
    const std::string s = "." + std::to_string(l);
    if (!(r = find("pred_wih" + s, 2, (uint64_t)PG4 * P, &p))) d.pred_w_ih[l] = (const uint16_t*)p;
    if (!r && !(r = find("pred_whh" + s, 2, (uint64_t)PG4 * P, &p))) d.pred_w_hh[l] = (const uint16_t*)p;
    if (!r && !(r = find("pred_bih" + s, 1, PG4, &p))) d.pred_b_ih[l] = (const float*)p;
    if (!r && !(r = find("pred_bhh" + s, 1, PG4, &p))) d.pred_b_hh[l] = (const float*)p;
  }
  if (!r && !(r = find("w1t", 2, (uint64_t)J * H, &p))) d.joint_w1t = (const uint16_t*)p;
  if (!r && !(r = find("w1p", 2, (uint64_t)J * P, &p))) d.joint_w1p = (const uint16_t*)p;
  if (!r && !(r = find("bt", 1, J, &p))) d.joint_bt = (const float*)p;
  if (!r && !(r = find("bp", 1, J, &p))) d.joint_bp = (const float*)p;
  if (!r && !(r = find("w2", 2, (uint64_t)NLAB * J, &p))) d.joint_w2 = (const uint16_t*)p;
  if (!r && !(r = find("b2", 1, NLAB, &p))) d.joint_b2 = (const float*)p;
  if (r) return r;
  // typed pointers into the image are aligned: the vector's storage comes from operator new
  // (>= 16-byte aligned) and every entry offset is a multiple of 64
  return rnnt_engine_create(&d, device, opts, out);
}

// The audio processor's file (tools/export_model.py --processor-file, rnnt_amd.featurizer.save_processor_file):
// fz_config fp32 [11] (the rnnt_featurizer_config fields in order), fz_window fp32 [win_length],
// fz_fb fp32 [nfilt][n_fft/2+1].  Replaces torch::jit::load of the TorchScript processor
// (csrc/rnnt_processor.hpp:17-22).
extern "C" int rnnt_featurizer_create_from_file(const char* path, int device, rnnt_featurizer** out) {
  if (!path || !out) return fail(RNNT_EINVAL, "null argument");
  *out = nullptr;
  PackFile pf;
  if (int r = pf.load(path)) return r;
  const void* p = nullptr;
  if (int r = pf.find("fz_config", 1, 11, &p)) return r;
  const float* c = (const float*)p;
  rnnt_featurizer_config cfg{};
  cfg.sample_rate = (int)c[0];
  cfg.n_fft = (int)c[1];
  cfg.win_length = (int)c[2];
  cfg.hop_length = (int)c[3];
  cfg.nfilt = (int)c[4];
  cfg.frame_splicing = (int)c[5];
  cfg.pad_out_feat = (int)c[6];
  cfg.preemph = c[7];
  cfg.dither = c[8];
  cfg.log_guard = c[9];
  cfg.norm_eps = c[10];
  const void* win = nullptr;
  const void* fb = nullptr;
  if (int r = pf.find("fz_window", 1, (uint64_t)cfg.win_length, &win)) return r;
  if (int r = pf.find("fz_fb", 1, (uint64_t)cfg.nfilt * (cfg.n_fft / 2 + 1), &fb)) return r;
  return rnnt_featurizer_create(&cfg, (const float*)win, (const float*)fb, device, out);
}

// ---- small utility kernels
__global__ void flen_kernel(const int32_t* lens, int32_t* flen, int n_pad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_pad) flen[i] = (lens[i] + 1) / 2;  // ceil(x_lens / stack_time_factor)
}
__global__ void stack_time_kernel(const int8_t* x, const int32_t* lens, int T, int n_pad, int C, int8_t* y) {
  const int tp = blockIdx.y, n = blockIdx.x;
  for (int i = threadIdx.x * 16; i < 2 * C; i += blockDim.x * 16) {
    const int half = i / C, t = 2 * tp + half, k = i % C;
    uint4 v = {0, 0, 0, 0};
    if (t < T && t < lens[n]) v = *(const uint4*)(x + ((size_t)t * n_pad + n) * C + k);
    *(uint4*)(y + ((size_t)tp * n_pad + n) * 2 * C + i) = v;
  }
}

// `stream` is used as given: 0 is the legacy default (null) stream, which is what torch's
// default stream is; the engine's own stream is only used by rnnt_engine_create.
static hipStream_t pick(rnnt_engine*, void* s) { return (hipStream_t)s; }

// state_ev protocol (see rnnt_engine::state_ev)
static int state_acquire(rnnt_engine* e, hipStream_t st) {
  if (e->pl_mode.load(std::memory_order_acquire))
    return fail(RNNT_EINVAL, "engine is in pipelined stream mode (rnnt_engine_encode_stream_pl)");
  if (e->state_rec && hipStreamWaitEvent(st, e->state_ev, 0) != hipSuccess)
    return fail(RNNT_EDEVICE, "hipStreamWaitEvent failed");
  return 0;
}
static int state_release(rnnt_engine* e, hipStream_t st) {
  if (hipEventRecord(e->state_ev, st) != hipSuccess) return fail(RNNT_EDEVICE, "hipEventRecord failed");
  e->state_rec = true;
  return 0;
}

// number of leading 128-row tiles that hold a row with len > thr
static int active_tiles(const std::vector<int>& tile_max, int thr) {
  int last = -1;
  for (int i = 0; i < (int)tile_max.size(); ++i)
    if (tile_max[i] > thr) last = i;
  return last + 1;
}

// Build the step job of encoder layer l at frame t (layers 0/1: feature frame, 2..4: stacked frame).
static EncStepArgs make_job(rnnt_engine* e, int l, int t, int n_pad, const int8_t* x, int mode, void* y, float* y32,
                            const int32_t* lens, int stacked_T) {
  const int I = ENC_I[l];
  EncStepArgs a{};
  a.W = e->enc_w[l];
  a.bq = e->enc_bq[l];
  a.x = x + (size_t)t * n_pad * I;
  a.h_in = e->h[l][(t + e->hpar[l]) & 1];
  a.h_out = e->h[l][(t + 1 + e->hpar[l]) & 1];
  a.c = e->c[l];
  a.I = I;
  a.mode = mode;
  a.rb = e->rb[l];
  a.in_s = e->in_s[l];
  a.out_s = e->out_s[l];
  a.lens = lens;
  if (mode == ENC_OUT_STACKED) {
    a.y8 = (int8_t*)y + (size_t)(t / 2) * n_pad * 2 * H;
    a.t = t;
    a.half = t & 1;
    a.zero_next = ((t & 1) == 0 && t + 1 == stacked_T);
  } else if (mode == ENC_OUT_I8) {
    a.y8 = (int8_t*)y + (size_t)t * n_pad * H;
  } else {
    a.y32 = y32 ? y32 + (size_t)t * n_pad * H : nullptr;
    a.fbf = (uint16_t*)y + (size_t)t * n_pad * H;
  }
  return a;
}

struct TickBuilder {
  EncTickArgs args{};
  int n = 0;
  // tiles: the job's active 128-row batch tiles, the leading `tiles` ones, or (mask != 0) the set
  // bits of mask
  void add(const EncStepArgs& a, int tiles, uint64_t mask = 0) {
    if (mask) tiles = __builtin_popcountll(mask);
    if (tiles <= 0) return;
    // keep jobs ordered by K descending (longest workgroups dispatched first)
    int p = n++;
    while (p > 0 && args.job[p - 1].I < a.I) {
      args.job[p] = args.job[p - 1];
      args.nbt[p] = args.nbt[p - 1];
      args.bmask[p] = args.bmask[p - 1];
      --p;
    }
    args.job[p] = a;
    args.nbt[p] = tiles;
    args.bmask[p] = mask;
  }
  int launch(rnnt_engine* e, hipStream_t st) {
    if (n == 0) return 0;
    args.njobs = n;
    e->step_launches++;
    return launch_lstm_i8_tick(args, st, e->tile) ? fail(RNNT_EDEVICE, "lstm tick launch failed") : 0;
  }
};

// One layer over T steps, one launch per step (op-level API).
static int run_layer(rnnt_engine* e, int l, int T, int n_pad, const int8_t* x, int mode, void* y, float* y32,
                     hipStream_t st) {
  for (int t = 0; t < T; ++t) {
    TickBuilder tb;
    tb.add(make_job(e, l, t, n_pad, x, mode, y, y32, nullptr, 0), n_pad / ENC_ROW_TILE);
    int r = tb.launch(e, st);
    if (r) return r;
  }
  return 0;
}

static int check_batch(rnnt_engine* e, int T, int n, int n_pad) {
  if (T <= 0 || T > e->opts.max_frames) return fail(RNNT_EINVAL, "T out of range");
  if (n <= 0 || n_pad < n || n_pad % ENC_PAD || n_pad > e->np_max)
    return fail(RNNT_EINVAL, "n / n_pad out of range (n_pad must be a multiple of 256 <= max_batch)");
  return 0;
}

static std::vector<int> tile_maxima(const int32_t* lens_host, int n, int n_pad) {
  std::vector<int> tm;
  if (!lens_host) return tm;
  tm.assign(n_pad / ENC_ROW_TILE, 0);
  for (int i = 0; i < n; ++i) tm[i / ENC_ROW_TILE] = std::max(tm[i / ENC_ROW_TILE], (int)lens_host[i]);
  return tm;
}

// Encoder state of the slots flagged in reset zeroed (PipelineState::update's masked_fill_ of
// pre/post hx and cx, metadata.cpp:120-131): workgroup (row, layer), 64 lanes x 16 B of h and c.
struct EncStateRows {
  int8_t* h[5];
  uint16_t* c[5];
};
__global__ void __launch_bounds__(64) enc_reset_rows_kernel(EncStateRows st, const int32_t* __restrict__ reset) {
  const int row = blockIdx.x, l = blockIdx.y;
  if (!reset[row]) return;
  const uint4 z = uint4{0u, 0u, 0u, 0u};
  *(uint4*)(st.h[l] + (size_t)row * H + threadIdx.x * 16) = z;
  *(uint4*)(st.c[l] + (size_t)row * H + threadIdx.x * 8) = z;
  *(uint4*)(st.c[l] + (size_t)row * H + 512 + threadIdx.x * 8) = z;
}

// The input of encode: an assembled [T][n_pad][256] fp32 batch, or the QSL's ragged sample store
// gathered in the quantize pass (store != nullptr).
struct EncInput {
  const float* feats = nullptr;
  const float* store = nullptr;
  const int64_t* offsets = nullptr;
};

// ---- persistent dataflow encode (lstm_i8_flow_kernel, encoder.hpp): the wavefront schedule's
// layer-steps as one launch's task list.  Used for small batches (n_pad <= 256) when the engine's
// tile setting is "flow" (or "auto", see flow_wanted).
static bool flow_wanted(const rnnt_engine* e, int n_pad) {
  (void)n_pad;  // any batch: the 128 x 128 task tile up to 256 rows, the 256 x 256 one beyond
  return e->tile == ENC_TILE_FLOW;
}

static int flow_alloc(rnnt_engine* e) {
  if (e->flow_dev) return 0;
  const size_t cap = 2 * (size_t)e->opts.max_frames + 3 * (size_t)e->tp_max + 8;
  const size_t bt = std::max<size_t>(ENC_FLOW_MAX_TILES, (size_t)e->np_max / ENC_FLOW_BIG_ROWS);  // blocks per step
  const size_t bytes = cap * sizeof(EncFlowStep) + cap * bt * sizeof(uint32_t);
  int r = dev_alloc(e, &e->flow_dev, bytes);
  if (!r) r = dev_alloc(e, &e->flow_ctr, cap + 4);
  if (r) return r;
  HIPCHK(hipHostMalloc((void**)&e->flow_host, bytes, hipHostMallocDefault));
  HIPCHK(hipHostMalloc((void**)&e->flow_abort, sizeof(uint32_t), hipHostMallocDefault));
  *e->flow_abort = 0;
  HIPCHK(hipEventCreateWithFlags(&e->flow_up_ev, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&e->flow_done_ev, hipEventDisableTiming));
  e->flow_cap = cap;
  return 0;
}

// the last flow launch's abort word, once its read-back has landed (non-blocking)
static int flow_poll(rnnt_engine* e) {
  if (!e->flow_check || hipEventQuery(e->flow_done_ev) != hipSuccess) return 0;
  e->flow_check = false;
  if (*e->flow_abort) {
    *e->flow_abort = 0;
    return fail(RNNT_EDEVICE, "encoder flow launch aborted: a task waited past its timeout (its outputs are invalid)");
  }
  return 0;
}

template <class Tiles>
static int run_flow(rnnt_engine* e, int T, int n_pad, const int32_t* lens, float* f_out, Tiles tiles, hipStream_t st) {
  int r = flow_alloc(e);
  if (r) return r;
  if (e->flow_up_pending) HIPCHK(hipEventSynchronize(e->flow_up_ev));  // the staging buffer is free again
  e->flow_up_pending = false;
  const int Tp = (T + 1) / 2;
  EncFlowStep* steps = (EncFlowStep*)e->flow_host;
  uint32_t* blocks = (uint32_t*)(e->flow_host + e->flow_cap * sizeof(EncFlowStep));
  std::vector<int> sid[5];  // step index of (layer, frame), -1: no tasks
  std::vector<int> snbt;
  for (int l = 0; l < 5; ++l) sid[l].assign(l < 2 ? T : Tp, -1);
  int ns = 0, nb = 0;
  const bool big = n_pad > ENC_FLOW_MAX_TILES * ENC_ROW_TILE;  // the 256 x 256 task tile
  const unsigned NGT = big ? ENC_FLOW_BIG_NGT : ENC_FLOW_NGT;
  const int max_nbt = big ? n_pad / ENC_FLOW_BIG_ROWS : ENC_FLOW_MAX_TILES;
  auto need = [&](int s) { return s < 0 ? 0u : NGT * (unsigned)snbt[s]; };
  struct Job { int l, t; EncStepArgs a; int nbt; };
  auto btiles = [&](int thr) { const int t = tiles(thr); return big ? (t + 1) / 2 : t; };  // task batch tiles
  const int n_ticks = std::max(T + 1, 2 * Tp + 4);
  for (int tau = 0; tau < n_ticks; ++tau) {
    Job jobs[5];
    int nj = 0;
    // the tick loop's jobs (encode_impl), ordered by K descending like TickBuilder
    if (tau < T) jobs[nj++] = {0, tau, make_job(e, 0, tau, n_pad, e->x0q, ENC_OUT_I8, e->yA, nullptr, lens, T), btiles(2 * (tau / 2))};
    if (tau >= 1 && tau - 1 < T)
      jobs[nj++] = {1, tau - 1, make_job(e, 1, tau - 1, n_pad, e->yA, ENC_OUT_STACKED, e->xs, nullptr, lens, T),
                    btiles(2 * ((tau - 1) / 2))};
    for (int l = 2; l < 5; ++l) {
      const int d = tau - (l + 1);
      if (d >= 0 && (d & 1) == 0 && d / 2 < Tp) {
        const int tp = d / 2;
        EncStepArgs a = l == 2   ? make_job(e, 2, tp, n_pad, e->xs, ENC_OUT_I8, e->yB, nullptr, lens, T)
                        : l == 3 ? make_job(e, 3, tp, n_pad, e->yB, ENC_OUT_I8, e->yC, nullptr, lens, T)
                                 : make_job(e, 4, tp, n_pad, e->yC, ENC_OUT_FINAL, e->fbf, f_out, lens, T);
        jobs[nj++] = {l, tp, a, btiles(2 * tp)};
      }
    }
    std::stable_sort(jobs, jobs + nj, [](const Job& x, const Job& y) { return x.a.I > y.a.I; });
    for (int j = 0; j < nj; ++j) {
      const Job& jb = jobs[j];
      if (jb.nbt <= 0) continue;
      if (jb.nbt > max_nbt || ns >= (int)e->flow_cap) return fail(RNNT_EINVAL, "flow encode: batch too large");
      // input frame: layer l-1 at the same frame (layer 2: the odd half of stacked frame t', i.e.
      // feature frame 2t'+1, or 2t' for an odd-T pad; its completion implies 2t''s); recurrent
      // state: layer l at t-1
      int dx = -1;
      if (jb.l == 1) dx = sid[0][jb.t];
      else if (jb.l == 2) dx = sid[1][std::min(2 * jb.t + 1, T - 1)];
      else if (jb.l > 2) dx = sid[jb.l - 1][jb.t];
      const int dh = jb.t > 0 ? sid[jb.l][jb.t - 1] : -1;
      EncFlowStep& s = steps[ns];
      s.a = jb.a;
      s.dep_x = dx;
      s.need_x = need(dx);
      s.dep_h = dh;
      s.need_h = need(dh);
      for (int nt = 0; nt < jb.nbt; ++nt) blocks[nb++] = (uint32_t)ns | ((uint32_t)nt << 16);
      sid[jb.l][jb.t] = ns++;
      snbt.push_back(jb.nbt);
    }
  }
  if (ns == 0) return 0;
  EncFlowArgs f{};
  f.steps = (const EncFlowStep*)e->flow_dev;
  f.blocks = (const uint32_t*)(e->flow_dev + e->flow_cap * sizeof(EncFlowStep));
  f.ctr = e->flow_ctr;
  f.n_steps = ns;
  f.n_tasks = nb * (int)NGT;
  f.timeout = 200000000ull;  // 2 s at 100 MHz: a config-3 encode takes a few ms
  HIPCHK(hipMemcpyAsync(e->flow_dev, e->flow_host, (size_t)ns * sizeof(EncFlowStep), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync((void*)f.blocks, blocks, (size_t)nb * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  HIPCHK(hipEventRecord(e->flow_up_ev, st));
  e->flow_up_pending = true;
  HIPCHK(hipMemsetAsync(e->flow_ctr, 0, ((size_t)ns + 2 + 3) / 4 * 16, st));
  static const int big_grid = [] {  // development knob: CUs the big-batch flow launch holds
    const char* v = dev_env("RNNT_ENC_FLOW_GRID");
    const int g = v ? atoi(v) : 256;
    return g >= 8 && g <= 256 ? g : 256;
  }();
  const int grid = std::min(f.n_tasks, big ? big_grid : 256);
  if (launch_lstm_i8_flow(f, grid, st, big)) return fail(RNNT_EDEVICE, "flow encode launch failed");
  HIPCHK(hipMemcpyAsync(e->flow_abort, e->flow_ctr + ns + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipEventRecord(e->flow_done_ev, st));
  e->flow_check = true;
  e->flow_launches++;
  e->step_launches++;
  return 0;
}

// reset == nullptr: a batch of whole utterances (every row's state starts at zero); otherwise a
// stream chunk (rnnt_engine_encode_stream): rows keep their state unless flagged.
static int encode_impl(rnnt_engine* e, const EncInput& in, const int32_t* lens, const int32_t* lens_host, int T, int n,
                       int n_pad, float* f_out, void* stream, const int32_t* reset = nullptr, bool pl = false) {
  if (!e || !lens || !(in.feats || (in.store && in.offsets))) return fail(RNNT_EINVAL, "null argument");
  if (e->enc_loaded != 0x1f) return fail(RNNT_EINVAL, "encoder weights not loaded");
  int r = check_batch(e, T, n, n_pad);
  if (r) return r;
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  if ((r = flow_poll(e))) return r;
  if (!pl && (r = state_acquire(e, st))) return r;
  const int Tp = (T + 1) / 2;
  const std::vector<int> tm = tile_maxima(lens_host, n, n_pad);
  if (!reset) {
    for (int l = 0; l < 5; ++l) {
      e->hpar[l] = 0;
      HIPCHK(hipMemsetAsync(e->h[l][0], 0, (size_t)n_pad * H, st));
      HIPCHK(hipMemsetAsync(e->c[l], 0, (size_t)n_pad * H * 2, st));
    }
  } else {
    EncStateRows sr;
    for (int l = 0; l < 5; ++l) {
      sr.h[l] = e->h[l][e->hpar[l] & 1];
      sr.c[l] = e->c[l];
    }
    hipLaunchKernelGGL(enc_reset_rows_kernel, dim3(n_pad, 5), dim3(64), 0, st, sr, reset);
    HIPCHK(hipGetLastError());
  }
  hipEvent_t ev0 = e->prof ? new_event(st) : nullptr;
  if (in.store ? launch_quantize_gather(in.store, in.offsets, lens, T, n, n_pad, e->in_s[0], e->x0q, st)
               : launch_quantize(in.feats, (int64_t)T * n_pad * FEAT, e->in_s[0], e->x0q, st))
    return fail(RNNT_EDEVICE, "quantize launch failed");
  // Wavefront schedule: tick tau runs layer 0 at frame tau, layer 1 at frame tau-1, and the
  // post_rnn layers 2/3/4 at stacked frame t' on ticks 2t'+3 / 2t'+4 / 2t'+5, i.e. as soon as
  // their inputs exist.  Every job of a tick is independent (inputs come from earlier ticks).
  const int nt_all = n_pad / ENC_ROW_TILE;
  auto tiles = [&](int thr) { return tm.empty() ? nt_all : active_tiles(tm, thr); };
  // stream chunks (unsorted slots): the tick skips every 128-row tile whose rows are all done at
  // this frame, not only a trailing run of them (a mask over at most 64 tiles; the set of active
  // tiles only shrinks with the frame, so a skipped tile's rows are finished for this call)
  const bool use_mask = reset != nullptr && !tm.empty() && nt_all <= 64 && !e->stream_prefix;
  auto tmask = [&](int thr) -> uint64_t {
    uint64_t m = 0;
    if (use_mask)
      for (int i = 0; i < nt_all; ++i)
        if (tm[i] > thr) m |= 1ull << i;
    return m;
  };
  constexpr int L4_LAG = 5;  // post_rnn layer 4 at stacked frame t' runs on tick 2t' + 5, right after layer 3
  const int n_ticks = flow_wanted(e, n_pad) ? 0 : std::max(T + 1, 2 * Tp + L4_LAG - 1);
  if (!n_ticks && (r = run_flow(e, T, n_pad, lens, f_out, tiles, st))) return r;
  for (int tau = 0; tau < n_ticks; ++tau) {
    TickBuilder tb;
    if (tau < T)
      tb.add(make_job(e, 0, tau, n_pad, e->x0q, ENC_OUT_I8, e->yA, nullptr, lens, T), tiles(2 * (tau / 2)), tmask(2 * (tau / 2)));
    if (tau >= 1 && tau - 1 < T) {
      const int t = tau - 1;
      tb.add(make_job(e, 1, t, n_pad, e->yA, ENC_OUT_STACKED, e->xs, nullptr, lens, T), tiles(2 * (t / 2)), tmask(2 * (t / 2)));
    }
    for (int l = 2; l < 5; ++l) {
      const int d = tau - (l == 4 ? L4_LAG : l + 1);  // = 2t'
      if (d >= 0 && (d & 1) == 0 && d / 2 < Tp) {
        const int tp = d / 2;
        if (l == 2) tb.add(make_job(e, 2, tp, n_pad, e->xs, ENC_OUT_I8, e->yB, nullptr, lens, T), tiles(2 * tp), tmask(2 * tp));
        if (l == 3) tb.add(make_job(e, 3, tp, n_pad, e->yB, ENC_OUT_I8, e->yC, nullptr, lens, T), tiles(2 * tp), tmask(2 * tp));
        if (l == 4) tb.add(make_job(e, 4, tp, n_pad, e->yC, ENC_OUT_FINAL, e->fbf, f_out, lens, T), tiles(2 * tp), tmask(2 * tp));
      }
    }
    if ((r = tb.launch(e, st))) return r;
  }
  hipLaunchKernelGGL(flen_kernel, dim3((n_pad + 255) / 256), dim3(256), 0, st, lens, e->flen, n_pad);
  HIPCHK(hipGetLastError());
  // every layer ran all its steps (layers 0/1: T frames, post_rnn: Tp stacked frames); rows of a
  // skipped tile are past their length in this call, i.e. finished
  for (int l = 0; l < 5; ++l) e->hpar[l] = (e->hpar[l] + (l < 2 ? T : Tp)) & 1;
  if (e->prof) e->ev_enc.push_back({ev0, new_event(st)});
  if (!pl && (r = state_release(e, st))) return r;
  e->encode_calls++;
  e->last_T = T;
  e->last_n = n;
  e->last_npad = n_pad;
  return 0;
}

extern "C" int rnnt_engine_encode(rnnt_engine* e, const float* feats, const int32_t* lens, const int32_t* lens_host,
                                  int T, int n, int n_pad, float* f_out, void* stream) {
  EncInput in;
  in.feats = feats;
  return encode_impl(e, in, lens, lens_host, T, n, n_pad, f_out, stream);
}

extern "C" int rnnt_engine_encode_gather(rnnt_engine* e, const float* store, const int64_t* offsets,
                                         const int32_t* lens, const int32_t* lens_host, int T, int n, int n_pad,
                                         float* f_out, void* stream) {
  if (!lens_host) return fail(RNNT_EINVAL, "encode_gather needs the host lengths");
  for (int i = 0; i < n; ++i)
    if (lens_host[i] < 0 || lens_host[i] > T) return fail(RNNT_EINVAL, "a length exceeds T");
  EncInput in;
  in.store = store;
  in.offsets = offsets;
  return encode_impl(e, in, lens, lens_host, T, n, n_pad, f_out, stream);
}

extern "C" int rnnt_engine_encode_stream(rnnt_engine* e, const float* store, const int64_t* offsets,
                                         const int32_t* lens, const int32_t* lens_host, const int32_t* reset, int T,
                                         int n, int n_pad, void* stream) {
  if (!lens_host || !reset) return fail(RNNT_EINVAL, "encode_stream needs the host lengths and the reset flags");
  for (int i = 0; i < n; ++i)
    if (lens_host[i] < 0 || lens_host[i] > T) return fail(RNNT_EINVAL, "a chunk length exceeds T");
  EncInput in;
  in.store = store;
  in.offsets = offsets;
  return encode_impl(e, in, lens, lens_host, T, n, n_pad, nullptr, stream, reset);
}

static int decode_impl(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res, void* stream,
                       const int32_t* reset);
extern "C" int rnnt_engine_decode(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res, void* stream) {
  return decode_impl(e, res, res_len, max_res, stream, nullptr);
}
extern "C" int rnnt_engine_decode_stream(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res,
                                         const int32_t* reset, void* stream) {
  if (!reset) return fail(RNNT_EINVAL, "decode_stream needs the reset flags");
  return decode_impl(e, res, res_len, max_res, stream, reset);
}

// The decode of one encoded batch / chunk: joint_trans of its final-layer output fbf (T frames
// before stacking, n rows of n_pad) with lengths flen, then the greedy loop; after_jt runs on the
// host right after joint_trans is enqueued (the pipelined hand-off point).
template <class AfterJT>
static int decode_core(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res, hipStream_t st,
                       const int32_t* reset, const uint16_t* fbf, const int32_t* flen, int T, int n, int n_pad,
                       AfterJT after_jt) {
  const int Tp = (T + 1) / 2;
  hipEvent_t ev0 = e->prof ? new_event(st) : nullptr;
  if (launch_joint_trans(e->dw, fbf, flen, e->F, Tp, n_pad, st))
    return fail(RNNT_EDEVICE, "joint_trans launch failed");
  hipEvent_t ev1 = e->prof ? new_event(st) : nullptr;
  int r = after_jt();
  if (r) return r;
  DecArgs a{};
  a.w = e->dw;
  a.F = e->F;
  a.f_lens = flen;
  a.hc = e->hc;
  a.G = e->G;
  a.PH = e->PH;
  a.res = res;
  a.res_len = res_len;
  a.N = n;
  a.Npad = n_pad;
  a.max_res = max_res;
  a.s = e->ds;
  a.max_iter = Tp * (MAXSYM + 1) + 2;  // every step emits or advances; <= 30 emits per frame
  a.persist_rows = e->persist_rows;
  const int steps = launch_greedy_decode(a, e->host_flags, e->poll_ev, st, reset);
  if (steps == -2)  // dec_persist_kernel needs its 48 + nj workgroups co-resident (rnnt_engine_set_decode_persist)
    return fail(RNNT_EDEVICE, "persistent decode timed out: its workgroups were not all resident (other kernels held "
                              "the CUs); turn the persistent tail off or give the engine the GPU");
  if (steps < 0) return fail(RNNT_EDEVICE, "greedy launch failed");
  e->decode_steps += steps;
  if (e->prof) e->ev_dec.push_back({ev0, ev1, new_event(st)});
  e->decode_calls++;
  return flow_poll(e);  // the greedy loop has synchronised with the encode: report an aborted flow launch
}

static int decode_impl(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res, void* stream,
                       const int32_t* reset) {
  if (!e || !res || !res_len) return fail(RNNT_EINVAL, "null argument");
  if (e->last_n <= 0) return fail(RNNT_EINVAL, "decode before encode");
  if (!e->xtab_ok || !e->joint1_loaded || !e->joint2_loaded)
    return fail(RNNT_EINVAL, "prediction (with embedding) / joint weights not loaded");
  if (max_res <= 0) return fail(RNNT_EINVAL, "max_res must be positive");
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  int r = state_acquire(e, st);
  if (r) return r;
  r = decode_core(e, res, res_len, max_res, st, reset, e->fbf, e->flen, e->last_T, e->last_n, e->last_npad,
                  [] { return 0; });
  return r ? r : state_release(e, st);
}

// ---- pipelined stream calls (see rnnt_engine::fbf_dec)
static int pl_init(rnnt_engine* e) {
  if (e->fbf_dec) return 0;
  const size_t NP = e->np_max, TPM = e->tp_max;
  int r = dev_alloc(e, &e->fbf_dec, TPM * NP * H);
  r = r ? r : dev_alloc(e, &e->flen_dec, NP);
  r = r ? r : dev_alloc(e, &e->flen_dpriv, NP);
  for (int i = 0; i < 2 && !r; ++i)
    if (hipEventCreateWithFlags(&e->pl_copy_ev[i], hipEventDisableTiming) != hipSuccess)
      r = fail(RNNT_EDEVICE, "hipEventCreate failed");
  if (!r && hipEventCreateWithFlags(&e->pl_handoff_ev, hipEventDisableTiming) != hipSuccess)
    r = fail(RNNT_EDEVICE, "hipEventCreate failed");
  return r;
}

extern "C" int rnnt_engine_encode_stream_pl(rnnt_engine* e, const float* store, const int64_t* offsets,
                                            const int32_t* lens, const int32_t* lens_host, const int32_t* reset,
                                            int T, int n, int n_pad, void* stream) {
  if (!e || !lens_host || !reset) return fail(RNNT_EINVAL, "encode_stream_pl needs the host lengths and the reset flags");
  for (int i = 0; i < n; ++i)
    if (lens_host[i] < 0 || lens_host[i] > T) return fail(RNNT_EINVAL, "a chunk length exceeds T");
  int r = 0;
  if (!e->pl_mode.load(std::memory_order_acquire)) {  // first pipelined call: after the earlier calls' work
    DEVICE_SCOPE(e->device);
    if ((r = pl_init(e)) || (r = state_acquire(e, pick(e, stream)))) return r;
    e->pl_mode.store(true, std::memory_order_release);
  }
  EncInput in;
  in.store = store;
  in.offsets = offsets;
  if ((r = encode_impl(e, in, lens, lens_host, T, n, n_pad, nullptr, stream, reset, true))) return r;
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  const int64_t k = e->pl_enc_k;
  {  // the decode side's buffers are free once chunk k-1's decode has handed them off
    std::unique_lock<std::mutex> lk(e->pl_mu);
    e->pl_cv.wait(lk, [&] { return e->pl_handoff_k >= k - 1 || e->pl_failed; });
    if (e->pl_failed) return fail(RNNT_EDEVICE, "an earlier pipelined decode_stream_pl failed");
  }
  if (k >= 1) HIPCHK(hipStreamWaitEvent(st, e->pl_handoff_ev, 0));
  const int Tp = (T + 1) / 2;
  HIPCHK(hipMemcpyAsync(e->fbf_dec, e->fbf, (size_t)Tp * n_pad * H * sizeof(uint16_t), hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpyAsync(e->flen_dec, e->flen, (size_t)n_pad * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
  HIPCHK(hipEventRecord(e->pl_copy_ev[k & 1], st));
  {
    std::lock_guard<std::mutex> lk(e->pl_mu);
    e->pl_meta[k & 1][0] = T;
    e->pl_meta[k & 1][1] = n;
    e->pl_meta[k & 1][2] = n_pad;
    e->pl_enc_k = k + 1;
  }
  return 0;
}

// a pipelined decode that cannot run marks the engine failed (sticky) and wakes the encode side,
// which then returns RNNT_EDEVICE instead of waiting for a hand-off that will not come
static int pl_fail(rnnt_engine* e, int code, const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(e->pl_mu);
    e->pl_failed = true;
  }
  e->pl_cv.notify_all();
  return fail(code, msg);
}

extern "C" int rnnt_engine_decode_stream_pl(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res,
                                            const int32_t* reset, void* stream) {
  if (!e) return fail(RNNT_EINVAL, "null engine");
  if (!e->pl_mode.load(std::memory_order_acquire)) return fail(RNNT_EINVAL, "decode_stream_pl before encode_stream_pl");
  if (!res || !res_len || !reset) return pl_fail(e, RNNT_EINVAL, "null argument");
  if (!e->xtab_ok || !e->joint1_loaded || !e->joint2_loaded)
    return pl_fail(e, RNNT_EINVAL, "prediction (with embedding) / joint weights not loaded");
  if (max_res <= 0) return pl_fail(e, RNNT_EINVAL, "max_res must be positive");
  const int64_t k = e->pl_dec_k;
  int T, n, n_pad;
  {
    std::unique_lock<std::mutex> lk(e->pl_mu);
    if (e->pl_failed) return fail(RNNT_EDEVICE, "an earlier pipelined decode_stream_pl failed");
    if (k >= e->pl_enc_k) {
      lk.unlock();
      return pl_fail(e, RNNT_EINVAL, "decode_stream_pl before its chunk's encode_stream_pl returned");
    }
    T = e->pl_meta[k & 1][0];
    n = e->pl_meta[k & 1][1];
    n_pad = e->pl_meta[k & 1][2];
  }
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  bool handed = false;
  auto hand_off = [&] {  // chunk k's inputs are consumed: encode k+1 may overwrite them
    handed = true;
    const bool ok = hipEventRecord(e->pl_handoff_ev, st) == hipSuccess;
    {
      std::lock_guard<std::mutex> lk(e->pl_mu);
      e->pl_handoff_k = k;
    }
    e->pl_cv.notify_all();
    return ok ? 0 : fail(RNNT_EDEVICE, "hipEventRecord failed");
  };
  int r = 0;
  if (hipStreamWaitEvent(st, e->pl_copy_ev[k & 1], 0) != hipSuccess ||
      hipMemcpyAsync(e->flen_dpriv, e->flen_dec, (size_t)n_pad * sizeof(int32_t), hipMemcpyDeviceToDevice, st) !=
          hipSuccess)
    r = fail(RNNT_EDEVICE, "stream wait / copy failed");
  if (!r) r = decode_core(e, res, res_len, max_res, st, reset, e->fbf_dec, e->flen_dpriv, T, n, n_pad, hand_off);
  if (!handed) hand_off();  // never leave the encode side waiting on a failed decode
  e->pl_dec_k = k + 1;
  if (r) {  // the chunk's results are not there: later chunks cannot continue its carried state
    const std::string msg = g_err;
    return pl_fail(e, r, msg);
  }
  return r;
}

extern "C" int rnnt_engine_set_profiling(rnnt_engine* e, int on) {
  if (!e) return fail(RNNT_EINVAL, "null engine");
  e->prof = on != 0;
  return 0;
}

extern "C" int rnnt_engine_get_stats(rnnt_engine* e, rnnt_stats* out, int reset) {
  if (!e || !out) return fail(RNNT_EINVAL, "null argument");
  DEVICE_SCOPE(e->device);
  memset(out, 0, sizeof(*out));
  for (auto& p : e->ev_enc) {
    float ms = 0;
    HIPCHK(hipEventSynchronize(p.second));
    HIPCHK(hipEventElapsedTime(&ms, p.first, p.second));
    out->encode_ms += ms;
  }
  for (auto& p : e->ev_dec) {
    float a = 0, b = 0;
    HIPCHK(hipEventSynchronize(p[2]));
    HIPCHK(hipEventElapsedTime(&a, p[0], p[1]));
    HIPCHK(hipEventElapsedTime(&b, p[1], p[2]));
    out->joint_trans_ms += a;
    out->greedy_ms += b;
  }
  out->step_launches = e->step_launches;
  out->decode_steps = e->decode_steps;
  out->encode_calls = e->encode_calls;
  out->decode_calls = e->decode_calls;
  if (reset) {
    for (auto& p : e->ev_enc) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
    for (auto& p : e->ev_dec) for (auto ev : p) (void)hipEventDestroy(ev);
    e->ev_enc.clear();
    e->ev_dec.clear();
    e->step_launches = e->decode_steps = e->encode_calls = e->decode_calls = 0;
  }
  return 0;
}

extern "C" int rnnt_engine_infer(rnnt_engine* e, const float* feats, const int32_t* lens, const int32_t* lens_host,
                                 int T, int n, int n_pad, int32_t* res, int32_t* res_len, int max_res, void* stream) {
  int r = rnnt_engine_encode(e, feats, lens, lens_host, T, n, n_pad, nullptr, stream);
  return r ? r : rnnt_engine_decode(e, res, res_len, max_res, stream);
}

extern "C" int rnnt_op_lstm_int8(rnnt_engine* e, int first, int count, const void* x, int T, int n_pad, int8_t* hx,
                                 uint16_t* cx, void* y, void* stream) {
  if (!e || !x || !hx || !cx || !y) return fail(RNNT_EINVAL, "null argument");
  if (first < 0 || count <= 0 || first + count > 5) return fail(RNNT_EINVAL, "bad layer range");
  if (T <= 0 || T > e->opts.max_frames || n_pad <= 0 || n_pad % ENC_PAD || n_pad > e->np_max)
    return fail(RNNT_EINVAL, "T / n_pad out of range");
  if (first <= 1 && first + count > 2) return fail(RNNT_EINVAL, "a call covers pre_rnn or post_rnn, not both");
  for (int l = first; l < first + count; ++l)
    if (!(e->enc_loaded >> l & 1)) return fail(RNNT_EINVAL, "encoder layer weights not loaded");
  if (first >= 2 && T > e->tp_max) return fail(RNNT_EINVAL, "post_rnn T exceeds ceil(max_frames/2)");
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  int r0 = state_acquire(e, st);
  if (r0) return r0;
  const int8_t* cur = (const int8_t*)x;
  if (first == 0) {
    if (launch_quantize((const float*)x, (int64_t)T * n_pad * FEAT, e->in_s[0], e->x0q, st))
      return fail(RNNT_EDEVICE, "quantize launch failed");
    cur = e->x0q;
  }
  for (int i = 0; i < count; ++i) {
    const int l = first + i;
    const size_t NH = (size_t)n_pad * H;
    e->hpar[l] = 0;
    HIPCHK(hipMemcpyAsync(e->h[l][0], hx + i * NH, NH, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(e->c[l], cx + i * NH, NH * 2, hipMemcpyDeviceToDevice, st));
    const bool last = (i == count - 1);
    int8_t* dst = last ? (int8_t*)y : ((cur == e->yA) ? e->yB : e->yA);
    int r;
    if (l == 4)
      r = run_layer(e, l, T, n_pad, cur, ENC_OUT_FINAL, e->fbf, (float*)y, st);
    else
      r = run_layer(e, l, T, n_pad, cur, ENC_OUT_I8, dst, nullptr, st);
    if (r) return r;
    HIPCHK(hipMemcpyAsync(hx + i * NH, e->h[l][T & 1], NH, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(cx + i * NH, e->c[l], NH * 2, hipMemcpyDeviceToDevice, st));
    cur = dst;
  }
  return state_release(e, st);
}

extern "C" int rnnt_op_stack_time(rnnt_engine* e, const int8_t* x, const int32_t* x_lens, int T, int n_pad, int C,
                                  int8_t* y, void* stream) {
  if (!e || !x || !x_lens || !y) return fail(RNNT_EINVAL, "null argument");
  if (T <= 0 || n_pad <= 0 || C <= 0 || C % 16) return fail(RNNT_EINVAL, "bad shape");
  DEVICE_SCOPE(e->device);
  hipLaunchKernelGGL(stack_time_kernel, dim3(n_pad, (T + 1) / 2), dim3(64), 0, pick(e, stream), x, x_lens, T, n_pad,
                     C, y);
  HIPCHK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- fp32 encoder (config 2)
static const int F32_I[5] = {240, 1024, 2048, 1024, 1024};   // real input widths
static const int F32_IP[5] = {256, 1024, 2048, 1024, 1024};  // padded to 32 (chain blocks)

extern "C" int rnnt_engine_load_f32_encoder(rnnt_engine* e, const float* const* wih, const float* const* whh,
                                            const float* const* bih, const float* const* bhh) {
  if (!e || !wih || !whh || !bih || !bhh) return fail(RNNT_EINVAL, "null argument");
  DEVICE_SCOPE(e->device);
  for (int l = 0; l < 5; ++l) {
    if (!wih[l] || !whh[l] || !bih[l] || !bhh[l]) return fail(RNNT_EINVAL, "null fp32 encoder weight");
    const int I = F32_I[l], Ip = F32_IP[l];
    std::vector<float> wi((size_t)G4 * Ip, 0.0f), wh((size_t)G4 * H), bi(G4), bh(G4);
    for (int g = 0; g < 4; ++g)
      for (int u = 0; u < H; ++u) {
        const int src = g * H + u, dst = 4 * u + g;  // gate-interleaved rows
        for (int k = 0; k < I; ++k) wi[(size_t)dst * Ip + chain_pos(k)] = wih[l][(size_t)src * I + k];
        for (int k = 0; k < H; ++k) wh[(size_t)dst * H + chain_pos(k)] = whh[l][(size_t)src * H + k];
        bi[dst] = bih[l][src];
        bh[dst] = bhh[l][src];
      }
    int r = load_buf(e, &e->f32_wih[l], wi);  // a reload overwrites in place
    if (!r) r = load_buf(e, &e->f32_whh[l], wh);
    if (!r) r = load_buf(e, &e->f32_bih[l], bi);
    if (!r) r = load_buf(e, &e->f32_bhh[l], bh);
    if (r) return r;
  }
  e->f32_loaded = true;
  return 0;
}

static int f32_workspace(rnnt_engine* e, int T, int n_pad) {
  if ((size_t)T <= e->f32_ws_T && (size_t)n_pad <= e->f32_ws_np) return 0;
  for (void* p : e->f32_ws) (void)hipFree(p);
  e->f32_ws.clear();
  const size_t Tp = (T + 1) / 2, NH = (size_t)n_pad * H;
  auto al = [&](float** p, size_t count) -> int {
    void* q = nullptr;
    if (hipMalloc(&q, count * sizeof(float) + 256) != hipSuccess) return fail(RNNT_ENOMEM, "hipMalloc failed (f32)");
    e->f32_ws.push_back(q);
    *p = (float*)q;
    return 0;
  };
  auto ali = [&](int32_t** p, size_t count) -> int {
    float* q = nullptr;
    const int rr = al(&q, count);
    *p = (int32_t*)q;
    return rr;
  };
  const size_t NP = (size_t)n_pad * P;
  int r = al(&e->f32_x, (size_t)T * n_pad * FEAT);
  if (!r) r = al(&e->f32_fc, Tp * NH);
  if (!r) r = al(&e->f32_F, Tp * n_pad * J);
  if (!r) r = ali(&e->f32_flen, n_pad);
  if (!r) r = al(&e->ds32.ph, 2 * NP);
  if (!r) r = al(&e->ds32.pc, 2 * NP);
  if (!r) r = al(&e->ds32.gh, 2 * NP);
  if (!r) r = al(&e->ds32.gc, 2 * NP);
  int32_t** ints[] = {&e->ds32.time, &e->ds32.added, &e->ds32.idx, &e->ds32.preg, &e->ds32.fin};
  for (auto pp : ints)
    if (!r) r = ali(pp, n_pad);
  if (!r) r = ali(&e->ds32.unfinished, 4);
  if (!r) r = al(&e->f32_ya, (size_t)T * NH);
  if (!r) r = al(&e->f32_xs, Tp * NH * 2);
  if (!r) r = al(&e->f32_yb, Tp * NH);
  if (!r) r = al(&e->f32_yc, Tp * NH);
  for (int l = 0; l < 5; ++l) {
    if (!r) r = al(&e->f32_h[l][0], NH);
    if (!r) r = al(&e->f32_h[l][1], NH);
    if (!r) r = al(&e->f32_c[l], NH);
  }
  if (r) {
    e->f32_ws_T = e->f32_ws_np = 0;
    return r;
  }
  e->f32_ws_T = T;
  e->f32_ws_np = n_pad;
  return 0;
}

// fp32 layer l's step at frame t (x / y advance by their per-frame strides); h ping-pongs by t
static EncF32StepArgs f32_job(rnnt_engine* e, int l, int t, int n, int n_pad, const float* x, int mode, float* y,
                              const int32_t* lens, int stacked_T) {
  const size_t NH = (size_t)n_pad * H;
  EncF32StepArgs a{};
  a.wih = e->f32_wih[l];
  a.whh = e->f32_whh[l];
  a.bih = e->f32_bih[l];
  a.bhh = e->f32_bhh[l];
  a.I = F32_I[l];
  a.Ip = F32_IP[l];
  a.x = x + (size_t)t * n_pad * a.Ip;
  a.h_in = e->f32_h[l][t & 1];
  a.h_out = e->f32_h[l][(t + 1) & 1];
  a.c = e->f32_c[l];
  a.n = n;
  a.mode = mode;
  a.lens = lens;
  if (mode == ENC_F32_STACKED) {
    a.y = y + (size_t)(t / 2) * NH * 2;
    a.t = t;
    a.half = t & 1;
    a.zero_next = ((t & 1) == 0 && t + 1 == stacked_T);
  } else {
    a.y = y ? y + (size_t)t * NH : nullptr;
    if (mode == ENC_F32_FINAL) {  // the decoders' copies of f: chain-permuted fp32, and bf16
      a.y2 = e->f32_fc + (size_t)t * NH;
      a.ybf = e->fbf && n_pad <= e->np_max && t < e->tp_max ? e->fbf + (size_t)t * NH : nullptr;
    }
  }
  return a;
}

extern "C" int rnnt_engine_encode_f32(rnnt_engine* e, const float* feats, const int32_t* lens, int T, int n, int n_pad,
                                      float* f_out, void* stream) {
  if (!e || !feats || !lens) return fail(RNNT_EINVAL, "null argument");
  if (!e->f32_loaded) return fail(RNNT_EINVAL, "fp32 encoder weights not loaded (rnnt_engine_load_f32_encoder)");
  if (T <= 0 || T > e->opts.max_frames || n <= 0 || n_pad < n || n_pad % 64)
    return fail(RNNT_EINVAL, "T / n / n_pad out of range (n_pad a multiple of 64)");
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  int r = state_acquire(e, st);
  if (r) return r;
  if ((r = f32_workspace(e, T, n_pad))) return r;
  const int Tp = (T + 1) / 2;
  if (launch_permute_feats(feats, (int64_t)T * n_pad, e->f32_x, st)) return fail(RNNT_EDEVICE, "permute launch failed");
  // Transcription.forward (modeling_rnnt.py:116-144): pre_rnn 2 layers -> StackTime -> post_rnn 3
  // layers, on the int8 path's wavefront schedule: tick tau runs layer 0 at frame tau, layer 1 at
  // tau-1 and post_rnn layer l at stacked frame t' on tick 2t' + l + 1 (encode_impl)
  const size_t NH = (size_t)n_pad * H;
  for (int l = 0; l < 5; ++l) {
    HIPCHK(hipMemsetAsync(e->f32_h[l][0], 0, NH * sizeof(float), st));
    HIPCHK(hipMemsetAsync(e->f32_c[l], 0, NH * sizeof(float), st));
  }
  const int n_ticks = std::max(T + 1, 2 * Tp + 4);
  for (int tau = 0; tau < n_ticks; ++tau) {
    EncF32TickArgs tk{};
    auto add = [&](const EncF32StepArgs& a) {  // keep jobs ordered by K descending
      int p = tk.njobs++;
      while (p > 0 && tk.job[p - 1].I < a.I) {
        tk.job[p] = tk.job[p - 1];
        --p;
      }
      tk.job[p] = a;
    };
    if (tau < T) add(f32_job(e, 0, tau, n, n_pad, e->f32_x, ENC_F32_NEXT, e->f32_ya, lens, T));
    if (tau >= 1 && tau - 1 < T) add(f32_job(e, 1, tau - 1, n, n_pad, e->f32_ya, ENC_F32_STACKED, e->f32_xs, lens, T));
    for (int l = 2; l < 5; ++l) {
      const int d = tau - (l + 1);  // = 2t'
      if (d < 0 || (d & 1) || d / 2 >= Tp) continue;
      const int tp = d / 2;
      if (l == 2) add(f32_job(e, 2, tp, n, n_pad, e->f32_xs, ENC_F32_NEXT, e->f32_yb, lens, Tp));
      if (l == 3) add(f32_job(e, 3, tp, n, n_pad, e->f32_yb, ENC_F32_NEXT, e->f32_yc, lens, Tp));
      if (l == 4) add(f32_job(e, 4, tp, n, n_pad, e->f32_yc, ENC_F32_FINAL, f_out, lens, Tp));
    }
    if (launch_lstm_f32_tick(tk, st)) return fail(RNNT_EDEVICE, "fp32 lstm tick launch failed");
  }
  // f_lens = ceil(lens / 2) for both decoders; the bf16 copy of f (written when the batch fits
  // the int8 workspace) lets rnnt_engine_decode run the f32 + enable_bf16 decoder on it
  hipLaunchKernelGGL(flen_kernel, dim3((n_pad + 255) / 256), dim3(256), 0, st, lens, e->f32_flen, n_pad);
  HIPCHK(hipGetLastError());
  e->last32_T = T;
  e->last32_n = n;
  e->last32_npad = n_pad;
  if (n_pad <= e->np_max && Tp <= e->tp_max) {
    hipLaunchKernelGGL(flen_kernel, dim3((n_pad + 255) / 256), dim3(256), 0, st, lens, e->flen, n_pad);
    HIPCHK(hipGetLastError());
    e->last_T = T;
    e->last_n = n;
    e->last_npad = n_pad;
  } else {
    e->last_n = 0;  // no bf16 copy: rnnt_engine_decode refuses until the next encode
  }
  return state_release(e, st);
}

// fp32 prediction LSTM weights (natural [1280][320] per layer, torch.nn.LSTM gate order) into the
// fp32 decoder's layout: gate-interleaved rows, chain-permuted k; reloads overwrite in place
static int load_f32_pred(rnnt_engine* e, const float* const* w_ih, const float* const* w_hh, const float* const* b_ih,
                         const float* const* b_hh) {
  auto mut = [](const float* q) { return const_cast<float*>(q); };
  for (int l = 0; l < 2; ++l) {
    if (!w_ih[l] || !w_hh[l] || !b_ih[l] || !b_hh[l]) return fail(RNNT_EINVAL, "null fp32 prediction weight");
    std::vector<float> wi((size_t)PG4 * P), wh((size_t)PG4 * P), bi(PG4), bh(PG4);
    for (int g = 0; g < 4; ++g)
      for (int u = 0; u < P; ++u) {
        const int src = g * P + u, dst = 4 * u + g;  // gate-interleaved rows
        for (int k = 0; k < P; ++k) {
          wi[(size_t)dst * P + chain_pos(k)] = w_ih[l][(size_t)src * P + k];
          wh[(size_t)dst * P + chain_pos(k)] = w_hh[l][(size_t)src * P + k];
        }
        bi[dst] = b_ih[l][src];
        bh[dst] = b_hh[l][src];
      }
    float *a = mut(e->dw32.wih[l]), *b = mut(e->dw32.whh[l]), *c = mut(e->dw32.bih[l]), *d = mut(e->dw32.bhh[l]);
    int r;
    if ((r = load_buf(e, &a, wi)) || (r = load_buf(e, &b, wh)) || (r = load_buf(e, &c, bi)) || (r = load_buf(e, &d, bh)))
      return r;
    e->dw32.wih[l] = a;
    e->dw32.whh[l] = b;
    e->dw32.bih[l] = c;
    e->dw32.bhh[l] = d;
  }
  e->f32_pred_loaded = true;
  return 0;
}

extern "C" int rnnt_engine_load_f32_prediction(rnnt_engine* e, const float* const* w_ih, const float* const* w_hh,
                                               const float* const* b_ih, const float* const* b_hh) {
  if (!e || !w_ih || !w_hh || !b_ih || !b_hh) return fail(RNNT_EINVAL, "null argument");
  DEVICE_SCOPE(e->device);
  return load_f32_pred(e, w_ih, w_hh, b_ih, b_hh);
}

extern "C" int rnnt_op_lstm_f32(rnnt_engine* e, const float* x, const float* hx, const float* cx, float* hy, float* cy,
                                int n_pad, void* stream) {
  if (!e || !x || !hx || !cx || !hy || !cy) return fail(RNNT_EINVAL, "null argument");
  if (!e->f32_pred_loaded) return fail(RNNT_EINVAL, "fp32 prediction weights not loaded (rnnt_engine_load_f32_prediction)");
  if (n_pad <= 0 || n_pad % 64) return fail(RNNT_EINVAL, "n_pad must be a positive multiple of 64");
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  const size_t NP = (size_t)n_pad * P;
  if (launch_op_lstm_f32(e->dw32, 0, x, hx, cx, hy, cy, n_pad, st) ||
      launch_op_lstm_f32(e->dw32, 1, hy, hx + NP, cx + NP, hy + NP, cy + NP, n_pad, st))
    return fail(RNNT_EDEVICE, "lstm_f32 launch failed");
  return 0;
}

extern "C" int rnnt_engine_load_f32_decoder(rnnt_engine* e, const rnnt_f32_decoder_desc* m) {
  if (!e || !m || !m->embed || !m->joint_w1t || !m->joint_w1p || !m->joint_bt || !m->joint_bp || !m->joint_w2 ||
      !m->joint_b2)
    return fail(RNNT_EINVAL, "null argument");
  DEVICE_SCOPE(e->device);
  std::vector<float> emb((size_t)29 * P, 0.0f);  // row 28: SOS (zero embedding)
  for (int g = 0; g < 28; ++g)
    for (int k = 0; k < P; ++k) emb[(size_t)g * P + chain_pos(k)] = m->embed[(size_t)g * P + k];
  // every buffer is allocated on the first load and overwritten in place by a reload (load_buf)
  auto mut = [](const float* q) { return const_cast<float*>(q); };
  float* p = mut(e->dw32.emb);
  int r = load_buf(e, &p, emb);
  if (r) return r;
  e->dw32.emb = p;
  if ((r = load_f32_pred(e, m->pred_w_ih, m->pred_w_hh, m->pred_b_ih, m->pred_b_hh))) return r;
  auto chained = [](const float* src, int rows, int rows_pad, int K) {
    std::vector<float> w((size_t)rows_pad * K, 0.0f);
    for (int i = 0; i < rows; ++i)
      for (int k = 0; k < K; ++k) w[(size_t)i * K + chain_pos(k)] = src[(size_t)i * K + k];
    return w;
  };
  float *w1t = mut(e->dw32.w1t), *w1p = mut(e->dw32.w1p), *bt = mut(e->dw32.bt), *bp = mut(e->dw32.bp),
        *w2 = mut(e->dw32.w2), *b2 = mut(e->dw32.b2);
  std::vector<float> b2v(NLAB_PAD, 0.0f);
  std::copy(m->joint_b2, m->joint_b2 + NLAB, b2v.begin());
  if ((r = load_buf(e, &w1t, chained(m->joint_w1t, J, J, H))) || (r = load_buf(e, &w1p, chained(m->joint_w1p, J, J, P))) ||
      (r = load_buf(e, &w2, chained(m->joint_w2, NLAB, NLAB_PAD, J))) ||
      (r = load_buf(e, &bt, std::vector<float>(m->joint_bt, m->joint_bt + J))) ||
      (r = load_buf(e, &bp, std::vector<float>(m->joint_bp, m->joint_bp + J))) || (r = load_buf(e, &b2, b2v)))
    return r;
  e->dw32.w1t = w1t;
  e->dw32.w1p = w1p;
  e->dw32.bt = bt;
  e->dw32.bp = bp;
  e->dw32.w2 = w2;
  e->dw32.b2 = b2;
  e->f32_dec_loaded = true;
  return 0;
}

extern "C" int rnnt_engine_decode_f32(rnnt_engine* e, int32_t* res, int32_t* res_len, int max_res, void* stream) {
  if (!e || !res || !res_len) return fail(RNNT_EINVAL, "null argument");
  if (!e->f32_dec_loaded) return fail(RNNT_EINVAL, "fp32 decoder weights not loaded (rnnt_engine_load_f32_decoder)");
  if (e->last32_n <= 0) return fail(RNNT_EINVAL, "decode_f32 before encode_f32");
  if (max_res <= 0) return fail(RNNT_EINVAL, "max_res must be positive");
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  int r = state_acquire(e, st);
  if (r) return r;
  const int Tp = (e->last32_T + 1) / 2;
  if (launch_f32_joint_trans(e->dw32, e->f32_fc, e->f32_F, Tp, e->last32_npad, st))
    return fail(RNNT_EDEVICE, "fp32 joint_trans launch failed");
  DecF32Args a{};
  a.w = e->dw32;
  a.s = e->ds32;
  a.F = e->f32_F;
  a.f_lens = e->f32_flen;
  a.res = res;
  a.res_len = res_len;
  a.N = e->last32_n;
  a.Npad = e->last32_npad;
  a.max_res = max_res;
  a.max_iter = Tp * (MAXSYM + 1) + 2;
  if (launch_greedy_decode_f32(a, e->host_flags, e->poll_ev, st) < 0) return fail(RNNT_EDEVICE, "fp32 greedy launch failed");
  return state_release(e, st);
}

// ---------------------------------------------------------------- operator-level decode
// torch.ops.intel_mlperf lstm_amx_bf16 / amx_linear_bf16_accum_relu / amx_linear_i16o32 /
// greedy_decode_update (reference models/modeling_rnnt.py:202, 269-283, 331-365) on the bound
// model, for the reference's op-by-op Python loop (models/decoder.py:171-212).
static int check_rows(int n_pad) { return n_pad > 0 && n_pad % 16 == 0; }

extern "C" int rnnt_op_lstm_bf16(rnnt_engine* e, const uint16_t* x, const uint16_t* hx, const float* cx, uint16_t* hy,
                                 float* cy, int n_pad, void* stream) {
  if (!e || !x || !hx || !cx || !hy || !cy) return fail(RNNT_EINVAL, "null argument");
  if (!check_rows(n_pad)) return fail(RNNT_EINVAL, "n_pad must be a positive multiple of 16");
  if (!e->pred_loaded) return fail(RNNT_EINVAL, "prediction weights not loaded");
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  const size_t NP = (size_t)n_pad * P;
  if (launch_op_lstm_bf16(e->dw, 0, x, hx, cx, hy, cy, n_pad, st) ||
      launch_op_lstm_bf16(e->dw, 1, hy, hx + NP, cx + NP, hy + NP, cy + NP, n_pad, st))
    return fail(RNNT_EDEVICE, "lstm_bf16 launch failed");
  return 0;
}

extern "C" int rnnt_op_joint_hidden(rnnt_engine* e, const float* f, const uint16_t* g, uint16_t* y1, int n_pad,
                                    void* stream) {
  if (!e || !f || !g || !y1) return fail(RNNT_EINVAL, "null argument");
  if (!check_rows(n_pad)) return fail(RNNT_EINVAL, "n_pad must be a positive multiple of 16");
  if (!e->joint1_loaded) return fail(RNNT_EINVAL, "joint linear1 weights not loaded");
  DEVICE_SCOPE(e->device);
  if (launch_op_joint_hidden(e->dw, f, g, y1, n_pad, pick(e, stream))) return fail(RNNT_EDEVICE, "joint launch failed");
  return 0;
}

extern "C" int rnnt_op_joint_logits(rnnt_engine* e, const uint16_t* y1, float* logits, int n_pad, void* stream) {
  if (!e || !y1 || !logits) return fail(RNNT_EINVAL, "null argument");
  if (!check_rows(n_pad)) return fail(RNNT_EINVAL, "n_pad must be a positive multiple of 16");
  if (!e->joint2_loaded) return fail(RNNT_EINVAL, "joint linear2 weights not loaded");
  DEVICE_SCOPE(e->device);
  if (launch_op_joint_logits(e->dw, y1, logits, n_pad, pick(e, stream))) return fail(RNNT_EDEVICE, "linear2 launch failed");
  return 0;
}

__global__ void op_count_unfinished_kernel(const int32_t* time_idx, const int32_t* f_lens, int n, int32_t* count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && time_idx[i] < f_lens[i]) atomicAdd(count, 1);
}

extern "C" int rnnt_op_greedy_update(rnnt_engine* e, const void* symbols, int symbols_i64, int32_t* symbols_added,
                                     int32_t* res, int32_t* res_idx, const float* f, int f_batch, const int32_t* f_lens,
                                     int32_t* time_idx, float* fi, int32_t* pre_g, uint16_t* const* pre_hg,
                                     float* const* pre_cg, const uint16_t* const* hg, const float* const* cg, int n,
                                     int max_res, void* stream) {
  if (!e || !symbols || !symbols_added || !res || !res_idx || !f || !f_lens || !time_idx || !fi || !pre_g || !pre_hg ||
      !pre_cg || !hg || !cg)
    return fail(RNNT_EINVAL, "null argument");
  for (int l = 0; l < 2; ++l)
    if (!pre_hg[l] || !pre_cg[l] || !hg[l] || !cg[l]) return fail(RNNT_EINVAL, "null state tensor");
  if (n <= 0 || f_batch < n || max_res <= 0) return fail(RNNT_EINVAL, "bad sizes");
  DEVICE_SCOPE(e->device);
  hipStream_t st = pick(e, stream);
  if (!e->op_count) {
    int r = dev_alloc(e, &e->op_count, 4);
    if (r) return r;
    HIPCHK(hipHostMalloc((void**)&e->op_count_host, sizeof(int32_t)));
  }
  int r = state_acquire(e, st);
  if (r) return r;
  GreedyUpdateArgs a{};
  a.symbols = symbols;
  a.sym64 = symbols_i64 != 0;
  a.symbols_added = symbols_added;
  a.res = res;
  a.res_idx = res_idx;
  a.f = f;
  a.f_batch = f_batch;
  a.f_lens = f_lens;
  a.time_idx = time_idx;
  a.fi = fi;
  a.pre_g = pre_g;
  for (int l = 0; l < 2; ++l) {
    a.pre_hg[l] = pre_hg[l];
    a.pre_cg[l] = pre_cg[l];
    a.hg[l] = hg[l];
    a.cg[l] = cg[l];
  }
  a.n = n;
  a.max_res = max_res;
  if (launch_op_greedy_update(a, st)) return fail(RNNT_EDEVICE, "greedy_update launch failed");
  HIPCHK(hipMemsetAsync(e->op_count, 0, sizeof(int32_t), st));
  hipLaunchKernelGGL(op_count_unfinished_kernel, dim3((n + 255) / 256), dim3(256), 0, st, time_idx, f_lens, n, e->op_count);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->op_count_host, e->op_count, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  if ((r = state_release(e, st))) return r;
  HIPCHK(hipStreamSynchronize(st));
  return *e->op_count_host == 0 ? 1 : 0;  // all(finish), the op's bool result
}

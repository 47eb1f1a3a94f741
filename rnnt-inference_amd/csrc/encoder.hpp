// encoder.hpp -- launch interface of the int8 encoder kernels (internal to the engine).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rnnt {

// Encoder workgroup tiles (encoder.hip): 256 gate rows x 256 batch rows (one workgroup per CU)
// or 128 x 128 (two per CU), chosen per tick; tick jobs count active batch rows in 128-row tiles.
constexpr int ENC_BATCH_TILE = 256;  // batch rows of the large tile
constexpr int ENC_ROW_TILE = 128;    // batch rows of the small tile = the granularity of EncTickArgs::nbt
constexpr int ENC_PAD = 256;         // batch buffers are padded to a multiple of this

// Packed row of (unit u, gate g) in the encoder weight image.  Each wave's 64 gate rows hold
// 16 units: MFMA tile i = u&3, lane group q = (u>>2)&3 and accumulator register g, i.e.
// row = 64*(u>>4) + 16*i + 4*q + g.  One lane then owns the four gates of units u0..u0+3
// (u0 = 16*(u>>4) + 4*q) for its batch row, so the cell epilogue reads/writes 4 consecutive
// units per access.
__host__ __device__ __forceinline__ int enc_packed_row(int u, int g) {
  return ((u >> 4) << 6) + ((u & 3) << 4) + (((u >> 2) & 3) << 2) + g;
}

enum EncOutMode { ENC_OUT_I8 = 0, ENC_OUT_STACKED = 1, ENC_OUT_FINAL = 2 };

struct EncStepArgs {
  const int8_t* W;     // packed [4096][I+1024], gate-interleaved rows
  const float* bq;     // packed [4096] cell bias terms B = (bq rb) * (4 | 8 for g) + 64
  const int8_t* x;     // this frame's input rows: [Npad][I]
  const int8_t* h_in;  // [Npad][1024] h_{t-1} (quantised with in_s)
  int8_t* h_out;       // [Npad][1024] h_t
  uint16_t* c;         // [Npad][1024] fp16 cell state, in place
  int8_t* y8;          // I8: [Npad][1024] frame rows; STACKED: [Npad][2048] stacked frame rows
  float* y32;          // FINAL: optional fp32 f rows [Npad][1024]
  uint16_t* fbf;     // FINAL: bf16 f rows [Npad][1024] (natural k, subnormals flushed): the joint's input
  const int32_t* lens; // [Npad] feature lengths (STACKED masking)
  int I;               // input width (256 / 1024 / 2048)
  int mode;            // EncOutMode
  int t;               // frame index (STACKED)
  int half;            // t % 2 (STACKED)
  int zero_next;       // STACKED: also zero the odd-T pad half
  float rb, in_s, out_s;
};

// One launch runs up to ENC_MAX_JOBS independent layer-steps (the wavefront schedule of
// engine.hip: layer l at its own frame), each over its leading nbt active batch tiles.
constexpr int ENC_MAX_JOBS = 5;
struct EncTickArgs {
  EncStepArgs job[ENC_MAX_JOBS];
  int nbt[ENC_MAX_JOBS];  // active 128-row batch tiles per job (leading tiles holding a row still running)
  // bmask[j] != 0: the job's active 128-row tiles are the set bits (any subset of the first 64
  // tiles; nbt[j] = its popcount) instead of the leading nbt[j] -- the Server's unsorted slots,
  // where a tile whose rows are all done in this chunk is skipped wherever it sits
  uint64_t bmask[ENC_MAX_JOBS];
  int njobs;
};
// the job's active batch tiles of a BN-row tile shape (BN = 128 or 256) as a mask over those tiles
__host__ __device__ inline uint64_t enc_tile_mask(uint64_t m128, int BN) {
  if (BN == 128) return m128;
  uint64_t m = 0;  // 256-row tile k = 128-row tiles 2k, 2k+1
  for (int k = 0; k < 32; ++k)
    if ((m128 >> (2 * k)) & 3ull) m |= 1ull << k;
  return m;
}

int launch_quantize(const float* feat, int64_t n, float s, int8_t* out, hipStream_t st);
// AssembleSamples + the layer-0 input quantizer in one pass: row i of the batch is the QSL sample
// stored at store[offsets[i] * 240 ...] (LoadSamplesToRam's [T_i][240] fp32 rows, ragged), frames
// t < lens[i]; out int8 [T][n_pad][256], zero past the length, in channels 240..255 and rows >= n.
int launch_quantize_gather(const float* store, const int64_t* offsets, const int32_t* lens, int T, int n, int n_pad,
                           float s, int8_t* out, hipStream_t st);
// tick tile shape: chosen per tick by the cost model (ENC_TILE_AUTO) or pinned (tests, sweeps);
// ENC_TILE_FLOW: a whole-call encode of a small batch runs as one persistent dataflow launch
// (lstm_i8_flow_kernel) instead of one launch per tick (the tick path treats it as AUTO)
enum { ENC_TILE_AUTO = 0, ENC_TILE_BIG = 1, ENC_TILE_SMALL = 2, ENC_TILE_TINY = 3, ENC_TILE_MINI = 5, ENC_TILE_FLOW = 6,
       ENC_TILE_TICKS = 7 };
int launch_lstm_i8_tick(const EncTickArgs& a, hipStream_t st, int forced = ENC_TILE_AUTO);

// ---- persistent dataflow encoder (small batches: at most ENC_FLOW_MAX_TILES active 128-row tiles)
// The wavefront schedule's layer-steps become tasks of one launch: task = (layer-step, 128-row gate
// tile, 128-row batch tile), dealt from a device queue in tick order; a task waits on per-step
// completion counters for its input frame (layer l-1) and its recurrent h (layer l at t-1), and
// publishes its outputs write-through before counting itself done.
constexpr int ENC_FLOW_NGT = 32;        // gate tiles per layer-step (the 128 x 128 tile)
constexpr int ENC_FLOW_MAX_TILES = 2;   // batch tiles (n_pad <= 256)
// Larger batches (development, RNNT_ENC_TILE=flow): the same dataflow launch over the 256 x 256 tile
// (16 gate tiles per layer-step, 256-row batch tiles), on RNNT_ENC_FLOW_GRID workgroups (default 256)
constexpr int ENC_FLOW_BIG_NGT = 16;
constexpr int ENC_FLOW_BIG_ROWS = 256;
struct EncFlowStep {
  EncStepArgs a;
  int dep_x, dep_h;       // step whose completion the input frame / the recurrent state needs (-1: none)
  unsigned need_x, need_h;  // its task count
};
struct EncFlowArgs {
  const EncFlowStep* steps;   // [n_steps], tick order
  const uint32_t* blocks;     // [n_tasks / ENC_FLOW_NGT]: step | batch tile << 16 (gate tile = task % NGT)
  uint32_t* ctr;              // [n_steps] done tasks, [n_steps] queue head, [n_steps + 1] abort flag
  int n_tasks, n_steps;
  unsigned long long timeout; // s_memrealtime ticks (100 MHz) one wait may spin before it aborts the launch
};
int launch_lstm_i8_flow(const EncFlowArgs& f, int grid, hipStream_t st, bool big = false);

}  // namespace rnnt

// emu_hip.hpp -- a host emulation of the HIP device model the decode kernels use, for finding
// indexing and logic errors on the CPU (tools/emu/build.sh; ASan catches out-of-bounds accesses
// because device buffers are plain host allocations).
//
// Model: a launch runs its workgroups one after another; a workgroup is blockDim.x host threads
// (one per lane) that meet at std::barrier for s_barrier, and wave-wide operations (ballot, shfl,
// MFMA) exchange values through a per-wave buffer between two wave barriers.  __shared__ becomes
// `static` (workgroups never overlap).  v_mfma_f32_16x16x32_bf16 is evaluated with the oracle's
// pinned MFMA accumulation model (oracle_mfma_bf16_dot), so results are bit-exact with the oracle.
// Development tool only: it is not part of the engine and never runs on the GPU path.
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <memory>
#include <ucontext.h>
#include <vector>
#include <tuple>
#include <algorithm>

extern "C" void oracle_mfma_bf16_dot(int N, int K, const float* acc, const float* a, const float* b, float* out);

#define __global__
#define __device__
#define __host__
#define __shared__ static
#define __forceinline__ inline
#define __launch_bounds__(...)

typedef int hipError_t;
enum { hipSuccess = 0, hipErrorNotReady = 600, hipErrorUnknown = 999 };
enum hipMemcpyKind { hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice, hipMemcpyDefault };
enum hipFuncAttribute { hipFuncAttributeMaxDynamicSharedMemorySize };
typedef void* hipStream_t;
typedef void* hipEvent_t;

struct dim3 {
  unsigned x, y, z;
  constexpr dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct uint4 { unsigned x, y, z, w; };
struct uint2 { unsigned x, y; };
struct int4 { int x, y, z, w; };
struct int2 { int x, y; };
struct float4 { float x, y, z, w; };
struct float2 { float x, y; };

struct EmuIdx { unsigned x, y, z; };
inline EmuIdx threadIdx{0, 0, 0};
inline EmuIdx blockIdx{0, 0, 0}, gridDim{1, 1, 1}, blockDim{1, 1, 1};

typedef float emu_v4f __attribute__((ext_vector_type(4)));

// ---- cooperative workgroup: one fiber per lane on one host thread
struct EmuBar {
  int members = 0, arrived = 0;
  unsigned gen = 0;
};
struct EmuWave {
  EmuBar bar;
  uint64_t v[64];
  uint16_t a[64][8], b[64][8];
};
struct EmuFiber {
  ucontext_t ctx;
  char* stack = nullptr;
  EmuBar* wait = nullptr;  // blocked at this barrier until its generation moves past wait_gen
  unsigned wait_gen = 0;
  bool done = false;
  void* asan_fake = nullptr;
};
struct EmuWG {
  EmuBar bar;
  std::vector<EmuWave> waves;
  std::vector<EmuFiber> fib;
  ucontext_t sched;
  void* sched_fake = nullptr;
  const void* sched_stack_bottom = nullptr;
  size_t sched_stack_size = 0;
};
inline EmuWG* emu_wg = nullptr;
inline int emu_tid = 0;
constexpr size_t EMU_STACK = 1 << 17;

#if defined(__has_feature)
#if __has_feature(address_sanitizer)
#define EMU_ASAN 1
#endif
#endif
#ifdef EMU_ASAN
extern "C" void __sanitizer_start_switch_fiber(void** fake_stack_save, const void* bottom, size_t size);
extern "C" void __sanitizer_finish_switch_fiber(void* fake_stack_save, const void** bottom_old, size_t* size_old);
#endif

// back to the scheduler (the fiber is blocked or finished)
inline void emu_yield() {
  EmuFiber& f = emu_wg->fib[emu_tid];
#ifdef EMU_ASAN
  __sanitizer_start_switch_fiber(f.done ? nullptr : &f.asan_fake, emu_wg->sched_stack_bottom, emu_wg->sched_stack_size);
#endif
  swapcontext(&f.ctx, &emu_wg->sched);
#ifdef EMU_ASAN
  __sanitizer_finish_switch_fiber(f.asan_fake, nullptr, nullptr);
#endif
}
inline void emu_arrive(EmuBar& b) {
  if (++b.arrived == b.members) {
    b.arrived = 0;
    ++b.gen;
    return;  // the last arriver goes on
  }
  EmuFiber& f = emu_wg->fib[emu_tid];
  f.wait = &b;
  f.wait_gen = b.gen;
  while (b.gen == f.wait_gen) emu_yield();
  f.wait = nullptr;
}
inline void emu_leave(EmuBar& b) {  // a lane that returned: later phases need one arrival less
  --b.members;
  if (b.members > 0 && b.arrived == b.members) {
    b.arrived = 0;
    ++b.gen;
  }
}
inline void emu_sync() { emu_arrive(emu_wg->bar); }
inline void __syncthreads() { emu_sync(); }
inline EmuWave& emu_wave() { return emu_wg->waves[emu_tid >> 6]; }

template <class T>
inline T emu_xchg(T v, int src_lane) {
  EmuWave& w = emu_wave();
  uint64_t u = 0;
  memcpy(&u, &v, sizeof(T));
  w.v[emu_tid & 63] = u;
  emu_arrive(w.bar);
  const uint64_t r = w.v[src_lane & 63];
  emu_arrive(w.bar);
  T out;
  memcpy(&out, &r, sizeof(T));
  return out;
}
template <class T> inline T __shfl(T v, int src) { return emu_xchg(v, src); }
template <class T> inline T __shfl_xor(T v, int m) { return emu_xchg(v, (emu_tid & 63) ^ m); }
inline unsigned long long __ballot(int pred) {
  EmuWave& w = emu_wave();
  w.v[emu_tid & 63] = pred ? 1 : 0;
  emu_arrive(w.bar);
  unsigned long long m = 0;
  for (int i = 0; i < w.bar.members && i < 64; ++i) m |= (w.v[i] & 1ull) << i;
  emu_arrive(w.bar);
  return m;
}
inline int __any(int pred) { return __ballot(pred) != 0; }
inline int __syncthreads_or(int pred) {
  static int acc = 0;
  emu_sync();
  if (emu_tid == 0) acc = 0;
  emu_sync();
  if (pred) acc = 1;
  emu_sync();
  const int r = acc;
  emu_sync();
  return r;
}

inline float emu_bf2f(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
// v_mfma_f32_16x16x32_bf16: lane l holds A[l%16][8(l/16)..+7], B[8(l/16)..+7][l%16] and
// D[4(l/16)+i][l%16]
template <class V>
inline emu_v4f emu_mfma_bf16(V a, V b, emu_v4f c) {
  static_assert(sizeof(V) == 16, "8 bf16");
  EmuWave& w = emu_wave();
  const int lane = emu_tid & 63;
  memcpy(w.a[lane], &a, 16);
  memcpy(w.b[lane], &b, 16);
  emu_arrive(w.bar);
  emu_v4f out;
  const int q = lane >> 4, col = lane & 15;
  for (int i = 0; i < 4; ++i) {
    const int row = 4 * q + i;
    float av[32], bv[32];
    for (int k = 0; k < 32; ++k) {
      av[k] = emu_bf2f(w.a[row + 16 * (k / 8)][k % 8]);
      bv[k] = emu_bf2f(w.b[col + 16 * (k / 8)][k % 8]);
    }
    const float ci = c[i];
    float o;
    oracle_mfma_bf16_dot(1, 32, &ci, av, bv, &o);
    out[i] = o;
  }
  emu_arrive(w.bar);
  return out;
}
#define __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B, C, x, y, z) emu_mfma_bf16(A, B, C)
// v_mfma_f32_16x16x4f32: lane l holds A[l%16][l/16], B[l/16][l%16], D[4(l/16)+i][l%16]; the four
// products are accumulated in k order (fmaf chain; DESIGN.md section 2, bit-identical on gfx950)
inline emu_v4f emu_mfma_f32_4(float a, float b, emu_v4f c) {
  EmuWave& w = emu_wave();
  const int lane = emu_tid & 63;
  float* fa = (float*)w.a[lane];
  float* fb = (float*)w.b[lane];
  fa[0] = a;
  fb[0] = b;
  emu_arrive(w.bar);
  emu_v4f out;
  const int q = lane >> 4, col = lane & 15;
  for (int i = 0; i < 4; ++i) {
    const int row = 4 * q + i;
    float acc = c[i];
    for (int k = 0; k < 4; ++k) acc = fmaf(((float*)w.a[row + 16 * k])[0], ((float*)w.b[col + 16 * k])[0], acc);
    out[i] = acc;
  }
  emu_arrive(w.bar);
  return out;
}
#define __builtin_amdgcn_mfma_f32_16x16x4f32(A, B, C, x, y, z) emu_mfma_f32_4(A, B, C)
// a wave barrier (lanes of a wave meet: the emulation has no implicit lockstep)
inline void emu_wave_sync() { emu_arrive(emu_wave().bar); }
#define __builtin_amdgcn_wave_barrier() emu_wave_sync()
#define __builtin_amdgcn_sched_barrier(x) ((void)0)
#define __builtin_amdgcn_s_setprio(x) ((void)0)
#define __builtin_amdgcn_s_memrealtime() 0ull
inline float emu_fmed3f(float a, float b, float c) { return fmaxf(fminf(a, b), fminf(fmaxf(a, b), c)); }
#define __builtin_amdgcn_fmed3f(a, b, c) emu_fmed3f(a, b, c)
inline uint32_t emu_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t s = (sel >> (8 * i)) & 0xff;
    uint32_t byte = s < 8 ? (uint32_t)(v >> (8 * s)) & 0xff : (s == 0x0c ? 0 : 0xff);
    r |= byte << (8 * i);
  }
  return r;
}
#define __builtin_amdgcn_perm(a, b, s) emu_perm(a, b, s)
template <class... A>
inline void emu_global_load_lds(A...) {
  fprintf(stderr, "emu: global_load_lds is not emulated\n");
  abort();
}
#define __builtin_amdgcn_global_load_lds(...) emu_global_load_lds(__VA_ARGS__)

inline int min(int a, int b) { return a < b ? a : b; }
inline int max(int a, int b) { return a > b ? a : b; }
inline float2 make_float2(float x, float y) { return float2{x, y}; }
inline int2 make_int2(int x, int y) { return int2{x, y}; }

inline unsigned int __float_as_uint(float f) { unsigned int u; memcpy(&u, &f, 4); return u; }
inline float __uint_as_float(unsigned int u) { float f; memcpy(&f, &u, 4); return f; }
inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }

template <class T, class U>
inline T atomicAdd(T* p, U v) { return __atomic_fetch_add(p, (T)v, __ATOMIC_SEQ_CST); }
template <class T, class U>
inline T atomicOr(T* p, U v) { return __atomic_fetch_or(p, (T)v, __ATOMIC_SEQ_CST); }

// runtime API over host memory
struct hipFuncAttributes {
  size_t sharedSizeBytes = 0;
};
inline hipError_t hipFuncGetAttributes(hipFuncAttributes* a, const void*) { a->sharedSizeBytes = 0; return hipSuccess; }
enum hipDeviceAttribute_t { hipDeviceAttributeMaxSharedMemoryPerMultiprocessor };
inline hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) { *v = 160 * 1024; return hipSuccess; }
inline const char* hipGetErrorString(hipError_t) { return "emu error"; }
inline hipError_t hipMalloc(void** p, size_t n) { *p = malloc(n ? n : 1); return *p ? hipSuccess : hipErrorUnknown; }
inline hipError_t hipFree(void* p) { free(p); return hipSuccess; }
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) { memcpy(d, s, n); return hipSuccess; }
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipFuncSetAttribute(const void*, hipFuncAttribute, int) { return hipSuccess; }
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t = nullptr) { memset(p, v, n); return hipSuccess; }
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t = nullptr) {
  memcpy(d, s, n);
  return hipSuccess;
}
inline hipError_t hipEventRecord(hipEvent_t, hipStream_t = nullptr) { return hipSuccess; }
inline hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
inline hipError_t hipEventQuery(hipEvent_t) { return hipSuccess; }  // launches run synchronously
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipDeviceSynchronize() { return hipSuccess; }
#define HIP_SYMBOL(x) (&(x))
inline hipError_t hipMemcpyFromSymbol(void* d, const void* sym, size_t n) { memcpy(d, sym, n); return hipSuccess; }
inline hipError_t hipMemcpyToSymbol(void* sym, const void* s, size_t n) { memcpy(sym, s, n); return hipSuccess; }

// a launch: workgroups in order, each as blockDim.x lane fibers scheduled round-robin
inline long emu_workgroups = 0;
inline std::vector<char*> emu_stacks;
template <class K, class... A>
struct EmuLaunch {
  K kern;
  std::tuple<A...> args;
};
template <class L>
inline void emu_fiber_main(unsigned lo, unsigned hi) {
  L* l = (L*)(((uintptr_t)hi << 32) | lo);
#ifdef EMU_ASAN
  __sanitizer_finish_switch_fiber(nullptr, &emu_wg->sched_stack_bottom, &emu_wg->sched_stack_size);
#endif
  std::apply(l->kern, l->args);
  const int t = emu_tid;
  emu_leave(emu_wg->waves[t >> 6].bar);
  emu_leave(emu_wg->bar);
  emu_wg->fib[t].done = true;
  emu_yield();  // never resumed
}
template <class K, class... A>
inline void emu_launch(K kern, dim3 g, dim3 b, A... args) {
  if (b.y != 1 || b.z != 1 || g.z != 1) {
    fprintf(stderr, "emu: 1-D blocks and 2-D grids only\n");
    abort();
  }
  const int nt = (int)b.x;
  gridDim = {g.x, g.y, g.z};
  blockDim = {b.x, 1, 1};
  using L = EmuLaunch<K, A...>;
  L l{kern, std::tuple<A...>(args...)};
  while ((int)emu_stacks.size() < nt) emu_stacks.push_back((char*)malloc(EMU_STACK));
  for (unsigned by = 0; by < g.y; ++by)
    for (unsigned bx = 0; bx < g.x; ++bx) {
      EmuWG wg;
      wg.bar.members = nt;
      wg.waves.resize((nt + 63) / 64);
      for (int w = 0; w < (int)wg.waves.size(); ++w) wg.waves[w].bar.members = std::min(64, nt - 64 * w);
      wg.fib.resize(nt);
      emu_wg = &wg;
      blockIdx = {bx, by, 0};
      const uintptr_t lp = (uintptr_t)&l;
      for (int t = 0; t < nt; ++t) {
        EmuFiber& f = wg.fib[t];
        getcontext(&f.ctx);
        f.stack = emu_stacks[t];
        f.ctx.uc_stack.ss_sp = f.stack;
        f.ctx.uc_stack.ss_size = EMU_STACK;
        f.ctx.uc_link = nullptr;
        makecontext(&f.ctx, (void (*)())emu_fiber_main<L>, 2, (unsigned)(lp & 0xffffffffu), (unsigned)(lp >> 32));
      }
      int alive = nt;
      while (alive > 0) {
        bool progress = false;
        for (int t = 0; t < nt; ++t) {
          EmuFiber& f = wg.fib[t];
          if (f.done || (f.wait && f.wait->gen == f.wait_gen)) continue;
          emu_tid = t;
          threadIdx = {(unsigned)t, 0, 0};
#ifdef EMU_ASAN
          __sanitizer_start_switch_fiber(&wg.sched_fake, f.stack, EMU_STACK);
#endif
          swapcontext(&wg.sched, &f.ctx);
#ifdef EMU_ASAN
          __sanitizer_finish_switch_fiber(wg.sched_fake, nullptr, nullptr);
#endif
          progress = true;
          if (f.done) --alive;
        }
        if (!progress) {
          fprintf(stderr, "emu: workgroup (%u, %u) deadlocked: %d lanes blocked at barriers\n", bx, by, alive);
          abort();
        }
      }
      emu_wg = nullptr;
      if (++emu_workgroups % 200 == 0 && getenv("EMU_PROGRESS")) fprintf(stderr, "emu: %ld workgroups\n", emu_workgroups);
    }
}
#define hipLaunchKernelGGL(K, G, B, S, ST, ...) emu_launch(K, dim3(G), dim3(B), __VA_ARGS__)

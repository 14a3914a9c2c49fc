// Internal definitions shared by the FIA HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "fia.h"

namespace fia {

constexpr int kWave = 64;
constexpr int kScoreThreads = 256;       // scoring workgroup
constexpr int kScoreRows = 4;            // related ratings per scoring thread
constexpr int kChunk = kScoreThreads * kScoreRows;   // related ratings per scoring chunk
constexpr int kPrepThreads = 256;        // Gram workgroup
constexpr int kSolveThreads = 64;        // one wave per query solve

// Device buffer with grow-on-demand capacity (never shrinks).
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  hipError_t reserve(size_t want) {
    if (want <= bytes) return hipSuccess;
    if (ptr) {
      // the old allocation may still be read by queued kernels
      hipError_t e = hipDeviceSynchronize();
      if (e != hipSuccess) return e;
      e = hipFree(ptr);
      if (e != hipSuccess) return e;
      ptr = nullptr;
      bytes = 0;
    }
    size_t cap = want < 256 ? 256 : want;
    hipError_t e = hipMalloc(&ptr, cap);
    if (e == hipSuccess) bytes = cap;
    return e;
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(ptr); }
};

// User-major (CSR) / item-major (CSC) rating index.  For side s the list of
// entity e is [ptr[e], ptr[e+1]); row = train row (ascending), other = the
// other endpoint's id, rating = train label.
struct Side {
  DevBuf ptr;     // int64 [n_entity + 1]
  DevBuf row;     // int32 [N]
  DevBuf other;   // int32 [N]
  DevBuf rating;  // float [N]
};

struct Index {
  int64_t N = 0, U = 0, I = 0;
  Side side[2];   // 0 = users (R_u), 1 = items (C_i)
  bool valid = false;
};

// Parameter table pointers (device, float32, owned by the caller).
struct Params {
  int model = -1, k = 0;
  int64_t U = 0, I = 0;
  const float* t[10] = {};
  double wd = 0.0, damping = 0.0;
  bool valid = false;
};

struct PhaseEvents {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[FIA_NUM_PHASES];
  std::vector<hipEvent_t> pool;
};

}  // namespace fia

struct fia_ctx {
  int device = 0;
  std::string err;
  fia::Params p;
  fia::Index idx;
  // per-entity Gram caches (packed lower triangle, fp64): [U * GS], [I * GS]
  fia::DevBuf gram[2];
  // NCF: per-entity layer-1 halves Pm*W1[:k] and Qm*W1[k:] (fp64) [U*k], [I*k]
  fia::DevBuf l1[2];
  bool prepared = false;
  // per-batch scratch
  fia::DevBuf rec;        // per-query scoring record (fp64)
  fia::DevBuf coff;       // int64 [Q+1] chunk offsets
  fia::DevBuf cquery;     // int32 [max chunks]
  fia::DevBuf cstart;     // int32 [max chunks]
  fia::DevBuf cand_pos;   // int32 [max chunks * K]
  fia::DevBuf cand_val;   // double [max chunks * K]
  fia::DevBuf scan_tmp;   // rocprim temporary storage
  fia::DevBuf flag;       // int32 [4] device status words
  fia::DevBuf nch;        // int64 [Q+1] chunk counts
  bool profiling = false;
  fia::PhaseEvents events;
};

namespace fia {

// ---- launchers implemented in the .hip units ----
hipError_t build_index(fia_ctx* c, int64_t N, int64_t U, int64_t I, const int32_t* user,
                       const int32_t* item, const float* rating, hipStream_t s, std::string& why);
hipError_t count_related(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi,
                         int64_t* offsets, hipStream_t s);
hipError_t write_related(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi,
                         const int64_t* offsets, int64_t* rel, hipStream_t s);
hipError_t build_chunks(fia_ctx* c, int64_t Q, const int64_t* offsets, int64_t max_chunks, hipStream_t s);
hipError_t exclusive_scan_i64(fia_ctx* c, const int64_t* in, int64_t* out, int64_t n, hipStream_t s);

// model kernels: return hipErrorInvalidValue-style codes, or set `unsupported`
hipError_t prepare_model(fia_ctx* c, hipStream_t s, bool& unsupported);
hipError_t query_model(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                       int64_t max_chunks, int64_t* rel_idx, double* influence, double* x_out, int K,
                       int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s,
                       bool& unsupported);
int model_num_params(int model, int k);
bool model_supported(int model, int k);

// phase event helpers (no-ops unless profiling)
void phase_begin(fia_ctx* c, int phase, hipStream_t s);
void phase_end(fia_ctx* c, int phase, hipStream_t s);

}  // namespace fia

#define FIA_HIP_TRY(expr)                       \
  do {                                          \
    hipError_t _e = (expr);                     \
    if (_e != hipSuccess) return _e;            \
  } while (0)

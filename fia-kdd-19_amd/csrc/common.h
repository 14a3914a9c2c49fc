// Internal definitions shared by the FIA HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "fia.h"

namespace fia {

constexpr int kWave = 64;
constexpr int kScoreThreads = 256;       // scoring workgroup (4 independent waves)
constexpr int kScoreRows = 4;            // related ratings per lane and chunk
constexpr int kChunk = 64 * kScoreRows;  // related ratings per scoring chunk (one wave)
constexpr int kRunQB = 16;               // queries per item-run block (k_score_mf_runs)
constexpr int kRunChunk = 128;           // related ratings per item-run descriptor (k_score_mf_runs)
constexpr int kNcfRunChunk = 64;         // ... for NCF k <= 16 (k_score_ncf_runs: one rating per lane)
constexpr int kRunUserCost = 3;          // scheduling cost of a user-side run descriptor (k_score_mf_runs
                                         // slices): 2 per descriptor + 1 per query of its run

// One scoring chunk: <= kChunk consecutive ratings of ONE side (user list or item
// list) of one query, so every value a wave needs from the query is wave-uniform.
struct ChunkDesc {
  int64_t list_base;   // index into the side's list arrays
  int64_t out_base;    // index into rel_idx / influence
  int32_t q;           // query
  int32_t pos0;        // related position of the chunk's first rating
  int32_t len;         // ratings in the chunk
  int32_t side;        // 0 = user list R_u, 1 = item list C_i
};
constexpr int kPrepThreads = 256;        // Gram workgroup
constexpr int kSolveThreads = 64;        // one wave per query solve
constexpr int kGramChunk = 256;          // list rows per Gram work item (MI355X sweep: 64/128/256/512)
constexpr int kGsSub = 16;              // ratings per Gram-stream sub-batch (4 f64 MFMA row-quads)
constexpr int kGsSlice = 256;           // longest Gram-stream segment (longer lists: partial slices;
                                        // <= 511: a segment's count rides in 9 bits of its descriptor)
constexpr int kGsTarget = 8;            // sub-batches per Gram-stream wave (a range closes at >= this)
// (ml-1m-ex same-box A/B, ms per step: target 16 0.1460-0.1461; 8 0.1446-0.1448; 32 0.1442-0.1453;
//  slices of 128 0.1483; at most 8 segments per range 0.1481)
constexpr uint32_t kGsNoRow = 0x7fffff00u;   // Gram-stream row offset of no rating: outside any
                                             // table's buffer range, even + a lane's column bytes
constexpr int kGsRing = 8;              // gathered sub-batches in the kernel's register ring
constexpr int kGsMaxSub = 48;           // most sub-batches of one wave's range (a multiple of kGsRing)
constexpr int kGsMaxSeg = 4;            // most segments (Grams) of one wave's range: staged in LDS,
                                        // stored when the range is done
constexpr int kMfmaQB = 16;             // queries per MF k in {32, 64} MFMA scoring work item
constexpr int kMfmaCPI = 4;             // list chunks per MFMA scoring work item
constexpr int kWgBlocks = 4;            // query blocks (one per wave) sharing a workgroup's gathered rows
constexpr int kQueryBlock = 8;           // queries per entity-shared scoring work item (small k; 16 measured no better)
static_assert(kGsSlice < 512, "a Gram-stream segment's count rides in 9 bits of its descriptor (out >> 23)");

// Device buffer with grow-on-demand capacity (never shrinks), allocated from the
// device's stream-ordered pool on the context's stream: growing a buffer frees the old
// block in stream order (kernels already queued on `s` still read it) and allocates
// the new one behind them -- no device-wide synchronisation on the query path.  Work
// queued on ANOTHER stream is covered by the ABI: a call arriving on a different stream
// than the context's previous call first synchronises the device (fia_ctx::stream,
// abi.hip enter_stream), so a stream-ordered free never overtakes a reader there.  A
// regrown buffer gets 25 % headroom so a slowly growing batch does not regrow it
// every call.  Contents are not preserved.
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  hipError_t reserve(size_t want, hipStream_t s) {
    if (want <= bytes && ptr) return hipSuccess;
    // a regrow inside a graph capture would free a block allocated outside the graph:
    // buffers must be sized by an eager call before capture
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      return hipErrorStreamCaptureUnsupported;
    size_t cap = want < 256 ? 256 : want;
    if (ptr) {
      const size_t grown = bytes + bytes / 4;
      if (grown > cap) cap = grown;
      hipError_t e = hipFreeAsync(ptr, s);
      if (e != hipSuccess) return e;
      ptr = nullptr;
      bytes = 0;
    }
    hipError_t e = hipMallocAsync(&ptr, cap, s);
    if (e == hipSuccess) bytes = cap; else ptr = nullptr;
    return e;
  }
  void release(hipStream_t s) {
    if (ptr) (void)hipFreeAsync(ptr, s);
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
  DevBuf order[2];  // int32 [n_entity]: entities by list length, longest first (Gram scheduling)
  // Gram work lists: items of <= kGramChunk list rows {entity, start, len, slot}; slot < 0 =
  // write the entity's Gram directly, else a partial slot summed (in slot order) by a combine
  // pass {entity, first_slot, n_slots, 0}
  DevBuf gitems[2], gcomb[2];
  int64_t n_gitems[2] = {0, 0}, n_gcomb[2] = {0, 0}, n_gslots[2] = {0, 0};
  // open-addressing set of train pairs: key u*I+i -> (#rows, sum of ratings); answers
  // "is the test pair itself a train row?" in O(1) for the Hessian's d2r term
  DevBuf pkey;    // uint64 [pcap], ~0 = empty
  DevBuf pcnt;    // int32  [pcap]
  DevBuf psum;    // double [pcap]
  int64_t pcap = 0;
  std::vector<int64_t> hptr[2];   // host copies of side[s].ptr (Gram work lists)
  std::vector<int32_t> hord[2];   // entities by list length, longest first (host)
  int64_t gchunk = 0;             // list rows per small-k Gram work item of gitems
  // MF k <= 16 Gram stream (build_gram_stream, k_gram_mf_stream): the lists of both sides cut
  // into sub-batches of kGsSub ratings, one descriptor each {meta, out} (meta = valid ratings
  // | last of its segment << 5 | side << 6 | dummy << 7 | entity << 8; out, on a segment's last
  // sub-batch: its rating count << 23 | partial slot + 1, 0 = the entity's own Gram), the byte
  // offsets of their other-side rows in stream order (kGsSub per sub-batch, kGsNoRow past a
  // list's end), and the first descriptor of every wave's range (whole lists up to kGsSlice
  // ratings, longer lists in kGsSlice slices whose partial Grams gscomb sums in slot order)
  DevBuf gsdesc, gsids, gswave, gscomb[2];
  int64_t n_gsw = 0, n_gsdesc = 0, n_gscomb[2] = {0, 0}, n_gsslots[2] = {0, 0};
  uint64_t gs_version = ~0ull;
  int gs_k = 0;
  uint64_t version = 0;           // bumped by every build_index
  bool valid = false;
};

// ---- device helpers shared by the kernels ----
constexpr unsigned long long kEmptyKey = ~0ull;

__host__ __device__ inline unsigned long long pair_hash(unsigned long long k) {
  k += 0x9e3779b97f4a7c15ull;
  k = (k ^ (k >> 30)) * 0xbf58476d1ce4e5b9ull;
  k = (k ^ (k >> 27)) * 0x94d049bb133111ebull;
  return k ^ (k >> 31);
}

struct PairTable {
  const unsigned long long* key;
  const int32_t* cnt;
  const double* sum;
  unsigned long long mask;
  __device__ inline void lookup(unsigned long long k, double& c, double& s) const {
    unsigned long long h = pair_hash(k) & mask;
    c = 0.0;
    s = 0.0;
    for (unsigned long long probe = 0; probe <= mask; ++probe) {
      unsigned long long kk = key[h];
      if (kk == k) { c = (double)cnt[h]; s = sum[h]; return; }
      if (kk == kEmptyKey) return;
      h = (h + 1) & mask;
    }
  }
  // the same lookup split in two: the first probe's load is issued early, the rest of the
  // chain (rarely more than one probe at load <= 1/2) resolves later
  __device__ inline void probe_start(unsigned long long k, unsigned long long& h, unsigned long long& kk) const {
    h = pair_hash(k) & mask;
    kk = key[h];
  }
  __device__ inline void probe_finish(unsigned long long k, unsigned long long h, unsigned long long kk, double& c,
                                      double& s) const {
    c = 0.0;
    s = 0.0;
    for (unsigned long long probe = 0; probe <= mask; ++probe) {
      if (kk == k) { c = (double)cnt[h]; s = sum[h]; return; }
      if (kk == kEmptyKey) return;
      h = (h + 1) & mask;
      kk = key[h];
    }
  }
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
  fia::DevBuf gpart[2];   // partial Grams of long lists (fp64, [n_gslots * GSP])
  bool prepared = false;
  // per-batch scratch
  fia::DevBuf rec;        // per-query scoring record (fp64)
  fia::DevBuf coff;       // int64 [Q+1] chunk offsets
  fia::DevBuf cdesc;      // ChunkDesc [max chunks]
  fia::DevBuf cand_pos;   // int32 [max chunks * K]
  fia::DevBuf cand_val;   // double [max chunks * K]
  fia::DevBuf qscan;      // k_query_scan tile words + counters (left zero by every launch)
  fia::DevBuf flag;       // int32 [4] device status words
  fia::DevBuf nch;        // int64 [Q+1] chunk counts
  fia::DevBuf coupled;    // int32 [Q + 1]: count, then queries whose test pair is a train row
  // query groups per entity (entity-shared scoring): global entity index g = e (users) or
  // U + e (items)
  fia::DevBuf gcnt;       // uint64 [U + I + 1] queries per entity -> exclusive scan in gstart
  fia::DevBuf gstart;     // int64 [U + I + 1]
  fia::DevBuf grank;      // int32 [2Q] rank of query q in its user group / item group
  fia::DevBuf gq;         // int32 [2Q] queries grouped by entity (users then items)
  fia::DevBuf qbase;      // int64 [2Q] per query and side: output base, candidate-slot base
  fia::DevBuf slices;     // int32 [n + 1] first descriptor of each equal-cost slice (k_score_mf_runs)
  fia::DevBuf wstart;     // int64 [U + I + 1] exclusive scan of the work items per entity
  fia::DevBuf gscan;      // k_group_scan tile words + counters (left zero by every launch)
  fia::DevBuf witems;     // int32 [3 * max items] {global entity, list chunk, query block}
  fia::DevBuf d1tab;      // NCF k <= 16: d1 per z2 ReLU mask [2^(k/2)][k] (fp64)
  // large-k path (bigk.hip): per-list-position entity, per-train-row residual / NCF backward
  // vectors, per-query Hessian inputs and solutions, solve lists and LDL^T scratch
  fia::DevBuf self[2];    // int32 [N] entity owning list position p of side s
  uint64_t self_version = ~0ull;
  fia::DevBuf resid;      // double [N]   e_j = r-hat_j - y_j by train row
                          //   (small-k NCF: [2][N] by list position of each side)
  fia::DevBuf gm[2];      // double [N*k] NCF g_mlp = W1_side . d1_j by train row, per side
                          //   (small-k NCF: [k][N] by list position)
  fia::DevBuf wfrag;      // large-k NCF: W2 / W1 as f64 MFMA B fragments [3 k^2] (k_ncf_wfrag)
  fia::DevBuf slot[2];    // int32 [n_entity] Gram cache slot (-1 = not cached) after fia_prepare_for
  fia::DevBuf mark;       // uint8 [U + I] entities referenced by the fia_prepare_for queries
  bool subset = false;    // caches cover only the fia_prepare_for entities (large-k models)
  bool small_subset = false;   // small k after fia_prepare_for: Grams of the `mark`ed entities only
  fia::DevBuf bitems[2], bcomb[2];   // large-k Gram work lists {entity, start, len, slot}
  int64_t n_bitems[2] = {0, 0}, n_bcomb[2] = {0, 0}, n_bslots[2] = {0, 0}, n_bcache[2] = {0, 0};
  uint64_t bitems_version = ~0ull;
  int bitems_k = 0;
  fia::DevBuf qwork;      // double [Q * QW] per-query n, dup terms, r-hat, v, theta
  fia::DevBuf xb;         // double [Q * 2 NPs] per-query solution (padded side blocks)
  fia::DevBuf syslist;    // int32 [1 + 2Q] {count, 2q + side ...} uncoupled side systems
  fia::DevBuf cpllist;    // int32 [1 + Q]  {count, q ...} coupled full systems
  fia::DevBuf lscr;       // double LDL^T factor scratch, one slab per resident solve workgroup
  int num_cus = 0;
  // the stream of the previous call (a switch synchronises first: DevBuf frees are ordered
  // on the calling stream only)
  hipStream_t stream = nullptr;
  bool has_stream = false;
  // small-k fia_prepare runs its Gram pass on `aux`, forked from the calling stream, so the
  // query-side scans of the next calls overlap it; the first consumer of the caches (the
  // solve of fia_query_batch, or any call that rewrites what the pass reads) joins `prep`
  hipStream_t aux = nullptr;
  hipEvent_t fork_ev = nullptr, prep_ev = nullptr;
  bool prep_pending = false;
  // NCF: the per-entity layer-1 rows (the first kernels of the pass), which the query-side MLP
  // prologue reads before the Gram caches are done
  hipEvent_t l1_ev = nullptr;
  bool l1_pending = false;
  unsigned profiling = 0;   // bit p: record phase p (fia_set_profiling)
  fia::PhaseEvents events;
  // the chunk-list scan's timing events when that phase is its one kernel (stamped by its
  // dispatch, no marker packets: query_impl sets them around build_chunks)
  hipEvent_t scan_ev[2] = {nullptr, nullptr};
};

namespace fia {

// ---- launchers implemented in the .hip units ----
hipError_t build_index(fia_ctx* c, int64_t N, int64_t U, int64_t I, const int32_t* user,
                       const int32_t* item, const float* rating, hipStream_t s, std::string& why);
hipError_t count_related(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi,
                         int64_t* offsets, hipStream_t s);
hipError_t write_related(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi,
                         const int64_t* offsets, int32_t* rel, hipStream_t s);
// per-query chunk offsets coff (+ chunk descriptors unless offsets_only; with `runs` the
// descriptors are the compacted work list of k_score_mf_runs: every user-side chunk, the
// item-side chunks of run heads only, their count at qbase[4Q]; and the equal-cost slices of
// that list, c->slices[0 .. n] with n at qbase[4Q + 1], slice_cost units each -- rounded up
// to a power of two)
hipError_t build_chunks(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                        int64_t max_chunks, bool offsets_only, hipStream_t s, int32_t* zero_word = nullptr,
                        bool runs = false, int slice_cost = 0, int run_chunk = kRunChunk);
hipError_t build_gram_lists(fia_ctx* c, int64_t chunk, hipStream_t s);
// the MF k <= 16 Gram stream of the current index (Index::gs*), rebuilt after build_index
hipError_t build_gram_stream(fia_ctx* c, int k, hipStream_t s);
// per-batch query groups + entity-chunk work items (needs build_chunks' coff first)
hipError_t build_groups(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                        int64_t max_items, int qb, hipStream_t s, int cpi = 1);

// model kernels: return hipErrorInvalidValue-style codes, or set `unsupported`
hipError_t prepare_model(fia_ctx* c, hipStream_t s, bool& unsupported);
// small k: caches of the queries' users and items only (fia_prepare_for); marks in c->mark
hipStream_t prepare_stream(fia_ctx* c, hipStream_t s);
hipError_t prepare_record(fia_ctx* c, hipStream_t ps, hipStream_t s);
hipError_t join_prepare(fia_ctx* c, hipStream_t s);
hipError_t join_l1(fia_ctx* c, hipStream_t s);
// fia_prepare_for, small k, in two calls: mark_only marks the queries' entities on s; then
// their Gram caches on ps
hipError_t prepare_model_for(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, hipStream_t s, hipStream_t ps,
                             bool& unsupported, bool mark_only);
hipError_t check_cover_small(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, int32_t* flag,
                             hipStream_t s);
hipError_t query_model(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                       int64_t max_chunks, int32_t* rel_idx, double* influence, double* x_out, int K,
                       int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s,
                       bool& unsupported,
                       const double* x_in = nullptr);
int model_num_params(int model, int k);
bool model_supported(int model, int k);

// large-k models (bigk.hip): MF k in {128, 256}, NCF k in {64, 128, 256}
bool big_supported(int model, int k);
hipError_t ensure_self(fia_ctx* c, hipStream_t s);   // c->self[s]: entity of each list position
// contexts alive on a device (abi.hip): > 1 means batches of several contexts share the GPU
int live_contexts(int device);
// qu == nullptr: caches for every entity; else only for the entities of the Q queries
hipError_t prepare_big(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, hipStream_t s);
// flag[2] |= 1 if a query's user or item has no cache after fia_prepare_for
hipError_t check_cover(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, int32_t* flag, hipStream_t s);
hipError_t query_big(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                     int64_t max_chunks, int32_t* rel_idx, double* influence, double* x_out, int K,
                     int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s,
                     const double* x_in = nullptr);
// MF k <= 16 item-run scoring (score_mf.hip); QueryArgs is in kern.h
// a one-kernel phase (scoring) timed by its own dispatch: the event pair goes to
// hipExtLaunchKernelGGL, which stamps the kernel's start and end from the dispatch packet
// (two marker packets around it idled the GPU ~5 us each); both null when not profiling
struct PhaseSpan {
  hipEvent_t a = nullptr, b = nullptr;
};
struct QueryArgs;
// MF k <= 16 Gram caches from the Gram stream (gram_mf.hip)
struct GramStreamArgs {
  const int2* desc;        // {meta, slot} per sub-batch (Index::gsdesc)
  const uint32_t* ids;     // other-side row byte offsets, kGsSub per sub-batch (quad-transposed)
  const int32_t* wave;     // first descriptor of each wave's range [n_waves + 1]
  int64_t n_waves;
  const float* emb_other[2];
  uint32_t bytes_other[2]; // their sizes (buffer ranges: a gather outside reads 0)
  double* gram[2];
  double* part[2];
  const uint8_t* mark;     // fia_prepare_for: entities to build (users [0, U), items [U, U + I)), or null
  int64_t moff[2];
};
hipError_t launch_gram_mf_stream(int k, const GramStreamArgs& G, hipStream_t s);
hipError_t launch_score_mf_runs(int k, int64_t grid, hipStream_t s, const QueryArgs& A, int64_t Q,
                                const ChunkDesc* cdesc, const int64_t* qbase, const int32_t* slices,
                                const double* rec, int32_t* rel_idx, double* influence, int K, int32_t* cand_pos,
                                double* cand_val, PhaseSpan ps);
// NCF k <= 16 item-run scoring (score_mf.hip)
hipError_t launch_score_ncf_runs(int k, int64_t grid, hipStream_t s, const QueryArgs& A, int64_t Q,
                                 const ChunkDesc* cdesc, const int64_t* qbase, const int32_t* slices,
                                 const double* rec, int32_t* rel_idx, double* influence, int K, int32_t* cand_pos,
                                 double* cand_val, PhaseSpan ps);
// MF k in {32, 64}, top-K <= 1 entity-shared f64-MFMA scoring (score_mfma.hip); full = both
// per-rating outputs present
hipError_t launch_score_mf_mfma(int k, bool full, int64_t grid, hipStream_t s, PhaseSpan ps, const QueryArgs& A,
                                int64_t nE, const int64_t* wstart, const int32_t* witems, const int64_t* gstart,
                                const int32_t* gq, const int64_t* qbase, const double* rec, int32_t* rel_idx,
                                double* influence, int K, int32_t* cand_pos, double* cand_val);
// per-query merge of chunk top-K candidates (models.hip); spc = candidate slot sets per chunk
hipError_t launch_topk_merge(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, int K, int spc,
                             int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s,
                             int64_t max_chunks);

// phase event helpers (no-ops unless profiling)
void phase_begin(fia_ctx* c, int phase, hipStream_t s);
void phase_end(fia_ctx* c, int phase, hipStream_t s);
PhaseSpan phase_span(fia_ctx* c, int phase);

}  // namespace fia

#define FIA_HIP_TRY(expr)                       \
  do {                                          \
    hipError_t _e = (expr);                     \
    if (_e != hipSuccess) return _e;            \
  } while (0)

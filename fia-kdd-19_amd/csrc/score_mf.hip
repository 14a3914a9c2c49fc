// MF k <= 16 scoring (the headline kernel of BASELINE config 2): item runs.
// Reference: influence_j = x . grad L(z_j) / n for every related rating j of a test
// rating (u, i) (src/influence/matrix_factorization.py:237-246), x = H_t^-1 v from the solve.
#include <cstdlib>

#include "kern.h"


namespace fia {

constexpr int kRunsWaves = 3;   // waves per SIMD the register budget is sized for
namespace {

// The wave's best (key, position, value) under the strict (key desc, position asc) order,
// in every lane: the wave max of the keys, then the smallest position among the lanes
// holding it (positions are unique among valid candidates, invalid lanes carry (-2,
// INT_MAX)), then that lane's value.  The same winner as wave_best with a third of the VALU
// (one f64 max and one i32 min per step instead of a full compare-and-select of the triple).
template <int CTRL>
__device__ __forceinline__ double dpp_max_f64(double m) {
  const long long b = __double_as_longlong(m);
  const int lo = dpp_i32<CTRL>((int)(b & 0xffffffffll)), hi = dpp_i32<CTRL>((int)(b >> 32));
  return fmax(m, __longlong_as_double(((long long)hi << 32) | (unsigned)lo));
}
template <bool SW32>
__device__ __forceinline__ double rows_max_f64(double m) {
  const long long b = __double_as_longlong(m);
  const unsigned lo = other_rows<SW32>((unsigned)(b & 0xffffffffll)), hi = other_rows<SW32>((unsigned)(b >> 32));
  return fmax(m, __longlong_as_double(((long long)hi << 32) | lo));
}
template <int CTRL>
__device__ __forceinline__ int dpp_min_i32(int p) {
  const int o = dpp_i32<CTRL>(p);
  return o < p ? o : p;
}
__device__ __forceinline__ void wave_top1(double& a, int& p, double& v) {
  double m = dpp_max_f64<0x128>(a);
  m = dpp_max_f64<0x124>(m);
  m = dpp_max_f64<0x122>(m);
  m = dpp_max_f64<0x121>(m);
  m = rows_max_f64<false>(m);
  m = rows_max_f64<true>(m);
  int pc = a == m ? p : 0x7fffffff;
  pc = dpp_min_i32<0x128>(pc);
  pc = dpp_min_i32<0x124>(pc);
  pc = dpp_min_i32<0x122>(pc);
  pc = dpp_min_i32<0x121>(pc);
  {
    const int o = (int)other_rows<false>((unsigned)pc);
    pc = o < pc ? o : pc;
  }
  {
    const int o = (int)other_rows<true>((unsigned)pc);
    pc = o < pc ? o : pc;
  }
  const unsigned long long who = __ballot(a == m && p == pc);
  const int l = who ? (int)__builtin_ctzll(who) : 0;
  const long long vb = __double_as_longlong(v);
  const int vlo = __builtin_amdgcn_readlane((int)(vb & 0xffffffffll), l), vhi = __builtin_amdgcn_readlane((int)(vb >> 32), l);
  v = __longlong_as_double(((long long)vhi << 32) | (unsigned)vlo);
  a = m;
  p = pc;
}

// k_score_mf_runs (MF k <= 16, the headline kernel).  A work descriptor is one chunk
// (<= kRunChunk = 128 consecutive ratings) of ONE side's list together with a RUN of
// consecutive batch queries sharing that side's entity (build_chunks runs mode: an item-side
// chunk is work only for the first query of a run of equal test items, <= kRunQB queries; a
// user-side chunk has a run of one).  A batch in item-major order -- the natural way to answer
// a test set -- shares each popular item's list across its queries without any group build;
// any order stays correct (runs of one).  The descriptor list is cut into slices of about
// equal cost (build_chunks: kRunUserCost per user-side descriptor, 2 + nq per item-side one),
// one one-wave workgroup per slice.  Per descriptor, one wave (2 ratings per lane):
//   * the list entries (other id, rating, train row) were loaded during the previous
//     descriptor; the chunk's other-side rows + biases are gathered ONCE (random 64-B rows
//     from the L2-resident tables) and converted to f64 once;
//   * e_j = theta_e . g_j + (b_e + g) + b_o - y_j ONCE per rating (it depends on the train
//     rating only: every query of the run has the same entity);
//   * per query of the run: its words by scalar loads from its record (x, 1/n, c_q, x_bias,
//     the test pair's other id, output / slot bases: wave-uniform, no VALU broadcasts),
//     s_j = x . g_j (16 f64 FMAs), influence, nontemporal stores of influence + train row,
//     the chunk's top-K candidates.
// Every load is unconditional (clamped indices): a load under a branch makes the compiler
// drain vmcnt(0) where the paths join.  The registers the query loop reads are produced by
// VALU (the f64 rows, 2 e_j) or passed through an empty asm (ids, rows), so the compiler's
// loop-preheader vmcnt flush does not wait for the next descriptor's list loads.
// raw buffer resource word 3 (gfx9 family) and the nontemporal cache-policy bit
constexpr int kBufWord3 = 0x00020000;
constexpr int kBufNT = 2;

struct RunArgs {
  const int32_t* other[2];
  const float* rating[2];
  const int32_t* row[2];
  const float* emb_other[2];    // side 0 (user lists R_u): the item table; side 1: the user table
  const float* bias_other[2];
};

// The chunk's best (key, position, value) for top-1, in every lane: each lane's best of its RT
// ratings (exact), then the wave max of the keys rounded to f32 (one DPP max per step); the
// lanes holding that f32 key are resolved exactly (one lane in practice; ties within an f32
// rounding step fall back to the exact f64 reduction).  Same winner as wave_best.
__device__ __forceinline__ float dpp_maxf(float x, float y) { return x > y ? x : y; }
template <int CTRL>
__device__ __forceinline__ float dpp_max_f32(float m) {
  return dpp_maxf(m, __int_as_float(dpp_i32<CTRL>(__float_as_int(m))));
}
__device__ __forceinline__ void wave_top1_fast(double& a, int& p, double& v) {
  // keys are |v| >= 0, -1 (NaN) or -2 (no candidate); f32 rounding keeps their order (weakly)
  const float k32 = (float)a;
  float m = dpp_max_f32<0x128>(k32);
  m = dpp_max_f32<0x124>(m);
  m = dpp_max_f32<0x122>(m);
  m = dpp_max_f32<0x121>(m);
  m = dpp_maxf(m, __int_as_float((int)other_rows<false>((unsigned)__float_as_int(m))));
  m = dpp_maxf(m, __int_as_float((int)other_rows<true>((unsigned)__float_as_int(m))));
  const unsigned long long who = __ballot(k32 == m);
  if (__builtin_expect(__popcll(who) == 1, 1)) {
    const int l = (int)__builtin_ctzll(who);
    const long long ab = __double_as_longlong(a), vb = __double_as_longlong(v);
    a = __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(ab >> 32), l) << 32) |
                             (unsigned)__builtin_amdgcn_readlane((int)(ab & 0xffffffffll), l));
    v = __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(vb >> 32), l) << 32) |
                             (unsigned)__builtin_amdgcn_readlane((int)(vb & 0xffffffffll), l));
    p = __builtin_amdgcn_readlane(p, l);
  } else {
    if (k32 != m) { a = -2.0; p = 0x7fffffff; }
    wave_best(a, p, v);
  }
}

// KM: 0 = no top-K, 1 = top-1, 2 = top-K for K_top > 1
template <class M, int KM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kRunsWaves))) void k_score_mf_runs(
    RunArgs A, int64_t Q, const ChunkDesc* __restrict__ cdesc, const int64_t* __restrict__ qbase,
    const int32_t* __restrict__ slices, const double* __restrict__ rec, int32_t* __restrict__ rel_idx,
    double* __restrict__ influence, int K_top, int32_t* __restrict__ cand_pos, double* __restrict__ cand_val) {
  static_assert(!M::ncf && M::K <= 16 && M::K % 4 == 0, "MF k in {8, 16}");
  constexpr int K = M::K, RT = kRunChunk / 64, NA = K / 4;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // bytes per rating of the two outputs (0: the caller passed NULL, include/fia.h)
  const int n_inf = influence ? 8 : 0, n_rel = rel_idx ? 4 : 0;
  // one equal-cost slice of the descriptor list per one-wave workgroup (build_chunks): the
  // hardware dispatcher hands slices to free wave slots, so the work is balanced at slice
  // granularity without atomics; the wave walks its slice's descriptors in order
  const int64_t nsl = qbase[4 * Q + 1];
  const int64_t sl = blockIdx.x;
  if (sl >= nsl) return;
  int64_t ch = slices[sl];
  const int64_t cend = slices[sl + 1];
  if (ch >= cend) return;
  (void)wave;
  // list entries of descriptor c (positions past the chunk's end clamped to its first entry)
  auto fetch = [&](int64_t c, int32_t (&o)[RT], float (&y)[RT], int32_t (&rw)[RT]) {
    const ChunkDesc dd = cdesc[c];
    const int sd = dd.side & 0xff;
    const int32_t* __restrict__ oth = A.other[sd] + dd.list_base;
    const float* __restrict__ rat = A.rating[sd] + dd.list_base;
    const int32_t* __restrict__ rr = A.row[sd] + dd.list_base;
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int idx = r * 64 + lane;
      const int li = idx < dd.len ? idx : 0;
      o[r] = oth[li];
      y[r] = rat[li];
      rw[r] = rr[li];
    }
  };
  int32_t o[RT], row[RT];
  float y[RT];
  fetch(ch, o, y, row);
  int64_t nx = ch + 1 < cend ? ch + 1 : -1;      // the next descriptor (-1: none)
  while (true) {
    const ChunkDesc d = cdesc[ch];
    const int sd = d.side & 0xff, nq = d.side >> 8;
    const int32_t q0 = d.q;
    const int len = d.len;
    // the chunk's gathers: other-side rows and biases
    float4 g4[RT][NA];
    float gb[RT];
    {
      const float* __restrict__ T = A.emb_other[sd];
      const float* __restrict__ bt = A.bias_other[sd];
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const float4* src = reinterpret_cast<const float4*>(T + (int64_t)o[r] * K);
#pragma unroll
        for (int c = 0; c < NA; ++c) g4[r][c] = src[c];
        gb[r] = bt[o[r]];
      }
    }
    // the next descriptor's list entries, behind the gathers (the last descriptor reloads
    // itself: no branch around the loads)
    const bool more = nx >= 0;
    int32_t no[RT], nrow[RT];
    float ny[RT];
    fetch(more ? nx : ch, no, ny, nrow);

    // rows to f64 (once per descriptor) and 2 e_j, from the run head's record: the entity's
    // own embedding a and b_e + g (scalar loads)
    double g[RT][K], e2[RT];
    {
      const double* __restrict__ Sh = rec + (int64_t)q0 * M::R + 4 + sd * M::SB;
      double av[K];
#pragma unroll
      for (int c = 0; c < K; ++c) av[c] = Sh[c];
      const double bias_s = Sh[2 * K];
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        double dot = 0.0;
#pragma unroll
        for (int c4 = 0; c4 < NA; ++c4) {
          g[r][4 * c4 + 0] = (double)g4[r][c4].x;
          g[r][4 * c4 + 1] = (double)g4[r][c4].y;
          g[r][4 * c4 + 2] = (double)g4[r][c4].z;
          g[r][4 * c4 + 3] = (double)g4[r][c4].w;
        }
#pragma unroll
        for (int c = 0; c < K; ++c) dot = fma(av[c], g[r][c], dot);
        e2[r] = 2.0 * (dot + bias_s + (double)gb[r] - (double)y[r]);
      }
    }
    // the loop reads ids / train rows through an asm: not "loaded" registers for the
    // compiler's preheader flush (which would wait for the next descriptor's list loads)
#pragma unroll
    for (int r = 0; r < RT; ++r) asm volatile("" : "+v"(o[r]), "+v"(row[r]));
    // the words of query q0 + j by scalar loads; the next query's are issued once this
    // query's are consumed (same registers) and land while its top-1 reduction runs
    struct Words {
      double x[K], inv_n, cq, xsb, dup;
      int64_t ou, oi, slot;
    };
    auto words = [&](int32_t qj) {
      Words w;
      const double* __restrict__ Rj = rec + (int64_t)qj * M::R;
      const double* __restrict__ Sj = Rj + 4 + sd * M::SB;
      const int64_t* __restrict__ qb = qbase + 4 * (int64_t)qj;
#pragma unroll
      for (int c = 0; c < K; ++c) w.x[c] = Sj[K + c];
      w.inv_n = Rj[0];
      w.cq = Rj[1];
      w.xsb = Sj[2 * K + 1];
      w.dup = Sj[2 * K + 2];
      w.ou = qb[0];
      w.oi = qb[1];
      w.slot = qb[2 + sd];
      return w;
    };
    Words wj = words(q0);
    int j = 0;
    do {
      const int32_t qj = q0 + j;
      const double* __restrict__ Rj = rec + (int64_t)qj * M::R;
      // two partial sums per rating (even / odd coordinates): 2 RT independent FMA chains
      double s[RT], s2[RT];
#pragma unroll
      for (int r = 0; r < RT; ++r) s[r] = s2[r] = 0.0;
#pragma unroll
      for (int c = 0; c < K; c += 2) {
        const double xc = wj.x[c], xd = wj.x[c + 1];
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          s[r] = fma(xc, g[r][c], s[r]);
          s2[r] = fma(xd, g[r][c + 1], s2[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < RT; ++r) s[r] += s2[r];
      const double inv_nj = wj.inv_n, cqj = wj.cq, xsbj = wj.xsb;
      const int32_t dupj = (int32_t)wj.dup;
      const int64_t ou = wj.ou, oi = wj.oi;
      const int64_t obj = sd ? oi : ou;
      double infl[RT];
      bool anyd = false;
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        infl[r] = (e2[r] * (s[r] + xsbj) + cqj) * inv_nj;
        anyd = anyd || (o[r] == dupj && r * 64 + lane < len);
      }
      if (__builtin_expect(__ballot(anyd) != 0, 0)) {
        // the test pair's own train row: e = r-hat(u,i) - y, s = x . v (as in the solve's
        // record), both of its copies in rel bit-identical
        const double xv = Rj[2], rhat_ui = Rj[3];
        const float* __restrict__ rat = A.rating[sd] + d.list_base;
#pragma unroll
        for (int r = 0; r < RT; ++r)
          if (o[r] == dupj && r * 64 + lane < len)
            infl[r] = (2.0 * (rhat_ui - (double)rat[r * 64 + lane]) * xv + cqj) * inv_nj;
      }
      const int32_t co = (int32_t)(d.out_base - (sd ? qbase[4 * (int64_t)q0 + 1] : qbase[4 * (int64_t)q0]));
      // buffer stores with the chunk's length as the range: lanes past it are dropped by the
      // hardware (no branch around the stores, so every query issues the same number of them
      // and the compiler's vmcnt waits for older loads stay exact); nt policy
      // (rel_idx / influence NULL -- a top-K-only call: ranges of 0 bytes drop every store; the
      // bases are formed as integers, never as pointer arithmetic on a null pointer)
      {
        const int64_t ob = obj + co;
        const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<double*>(reinterpret_cast<uintptr_t>(influence) + (uintptr_t)ob * 8), 0, len * n_inf, kBufWord3);
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<int32_t*>(reinterpret_cast<uintptr_t>(rel_idx) + (uintptr_t)ob * 4), 0, len * n_rel, kBufWord3);
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          const int idx = r * 64 + lane;
          const long long ib = __double_as_longlong(infl[r]);
          __builtin_amdgcn_raw_buffer_store_b64(
              (__attribute__((ext_vector_type(2))) unsigned){(unsigned)(ib & 0xffffffffll), (unsigned)(ib >> 32)}, ri,
              idx * 8, 0, kBufNT);
          __builtin_amdgcn_raw_buffer_store_b32((unsigned)row[r], rr, idx * 4, 0, kBufNT);
        }
      }
      const int64_t slot = wj.slot + co / kRunChunk;
      const int32_t pbj = sd ? (int32_t)(oi - ou) : 0;
      wj = words(j + 1 < nq ? qj + 1 : qj);
      if constexpr (KM != 0) {
        if constexpr (KM == 1) {
          // the lane's best over its rows (positions ascend with r), then the wave's
          double ba = -2.0, bv = 0.0;
          int bp = 0x7fffffff;
#pragma unroll
          for (int r = 0; r < RT; ++r) {
            const int idx = r * 64 + lane;
            const double key = idx < len ? topk_key(infl[r]) : -2.0;
            if (key > ba) { ba = key; bp = idx; bv = infl[r]; }
          }
          wave_top1_fast(ba, bp, bv);
          // lane 0 stores the slot: a one-element buffer range drops the other lanes (no branch)
          const bool okk = ba > -1.5;
          const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(cand_pos + slot, 0, 4, kBufWord3);
          const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(cand_val + slot, 0, 8, kBufWord3);
          const long long vb = __double_as_longlong(okk ? bv : (double)NAN);
          __builtin_amdgcn_raw_buffer_store_b32((unsigned)(okk ? pbj + co + bp : -1), rp, lane * 4, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b64(
              (__attribute__((ext_vector_type(2))) unsigned){(unsigned)(vb & 0xffffffffll), (unsigned)(vb >> 32)}, rv,
              lane * 8, 0, 0);
        } else {
          double ca[RT];
          int cp[RT];
#pragma unroll
          for (int r = 0; r < RT; ++r) {
            const int idx = r * 64 + lane;
            const bool ok = idx < len;
            cp[r] = ok ? pbj + co + idx : -1;
            ca[r] = ok ? topk_key(infl[r]) : -2.0;
          }
          double pa = INFINITY;
          int pp = -1;
          for (int t = 0; t < K_top; ++t) {
            double ba = -2.0, bv = 0.0;
            int bp = 0x7fffffff;
#pragma unroll
            for (int r = 0; r < RT; ++r)
              if (cp[r] >= 0 && better(pa, pp, ca[r], cp[r]) && better(ca[r], cp[r], ba, bp)) {
                ba = ca[r]; bp = cp[r]; bv = infl[r];
              }
            wave_best(ba, bp, bv);
            if (lane == 0) {
              const bool okk = ba > -1.5;
              cand_pos[slot * K_top + t] = okk ? bp : -1;
              cand_val[slot * K_top + t] = okk ? bv : NAN;
            }
            pa = ba;
            pp = bp;
          }
        }
      }
    } while (++j < nq);
    if (!more) break;
    ch = nx;
    nx = ch + 1 < cend ? ch + 1 : -1;
#pragma unroll
    for (int r = 0; r < RT; ++r) { o[r] = no[r]; y[r] = ny[r]; row[r] = nrow[r]; }
  }
}

// ------------------------------------------------------------------------------------
// k_score_ncf_runs (NCF k <= 16: BASELINE config 3).  The item-run schedule of k_score_mf_runs
// for NCF (ncf:193-280): descriptor = a chunk of <= kNcfRunChunk = 64 ratings of one side's
// list + the run of consecutive batch queries sharing that side's entity, one rating per lane
// (yelp-ex lists hold ~24 ratings: the entity-shared k_score_ncf scored 4 rows per lane and
// left ~60 % of its lanes idle, after a group build).  Per rating, once per descriptor: the
// list entries, e_j and the two ReLU masks the Gram pass stored per list position, d1_j =
// 1[z1 > 0] * T[z2 mask] (k_ncf_d1_table, an L1-resident row) and the other side's gmf row;
// per query of the run its words by scalar loads (y = W1_side^T x_mlp after k_ncf_rec_y,
// W3g * x_gmf, the test pair's other id, the header): s_jq = y . d1_j + (W3g x_gmf) . gmf_o,
// influence, raw buffer stores ranged to the chunk (rel_idx / influence NULL: ranges of 0),
// the chunk's top-K candidates.
// ------------------------------------------------------------------------------------
struct NcfRunArgs {
  const int32_t* other[2];
  const float* rating[2];
  const int32_t* row[2];
  const int32_t* mask[2];      // per list position: bits [0, k) z1 > 0, [k, 3k/2) z2 > 0
  const double* resid;         // e_j per list position [side][N]
  const float* gmf_other[2];   // side 0 (user lists): the item gmf table; side 1: the user gmf table
  const double* d1tab;         // [2^(k/2)][k]
  int64_t N;
};

template <class M, int KM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kRunsWaves))) void k_score_ncf_runs(
    NcfRunArgs A, int64_t Q, const ChunkDesc* __restrict__ cdesc, const int64_t* __restrict__ qbase,
    const int32_t* __restrict__ slices, const double* __restrict__ rec, int32_t* __restrict__ rel_idx,
    double* __restrict__ influence, int K_top, int32_t* __restrict__ cand_pos, double* __restrict__ cand_val) {
  static_assert(mask_path<M>() && M::K % 4 == 0, "NCF k in {8, 16}");
  constexpr int K = M::K, NA = K / 4, CH = kNcfRunChunk;
  static_assert(CH == 64, "one rating per lane");
  const int lane = threadIdx.x & 63;
  const int n_inf = influence ? 8 : 0, n_rel = rel_idx ? 4 : 0;
  const int64_t nsl = qbase[4 * Q + 1];
  const int64_t sl = blockIdx.x;
  if (sl >= nsl) return;
  int64_t ch = slices[sl];
  const int64_t cend = slices[sl + 1];
  if (ch >= cend) return;
  // list entries of descriptor c (lanes past the chunk's end clamped to its first entry)
  auto fetch = [&](int64_t c, int32_t& o, float& y, int32_t& rw, double& e, int32_t& mk) {
    const ChunkDesc dd = cdesc[c];
    const int sd = dd.side & 0xff;
    const int64_t p = dd.list_base + (lane < dd.len ? lane : 0);
    o = A.other[sd][p];
    y = A.rating[sd][p];
    rw = A.row[sd][p];
    e = A.resid[sd * A.N + p];
    mk = A.mask[sd][p];
  };
  int32_t o, row, mk;
  float y;
  double e;
  fetch(ch, o, y, row, e, mk);
  int64_t nx = ch + 1 < cend ? ch + 1 : -1;
  while (true) {
    const ChunkDesc d = cdesc[ch];
    const int sd = d.side & 0xff, nq = d.side >> 8;
    const int32_t q0 = d.q;
    const int len = d.len;
    // the rating's gathers: the other side's gmf row and its d1 table row
    float4 g4[NA];
    double2 t2[K / 2];
    {
      const float4* src = reinterpret_cast<const float4*>(A.gmf_other[sd] + (int64_t)o * K);
#pragma unroll
      for (int c = 0; c < NA; ++c) g4[c] = src[c];
      const double2* tr = reinterpret_cast<const double2*>(A.d1tab + (int64_t)(mk >> K) * K);
#pragma unroll
      for (int c = 0; c < K / 2; ++c) t2[c] = tr[c];
    }
    const bool more = nx >= 0;
    int32_t no, nrow, nmk;
    float ny;
    double ne;
    fetch(more ? nx : ch, no, ny, nrow, ne, nmk);
    double g[K], d1[K];
#pragma unroll
    for (int c4 = 0; c4 < NA; ++c4) {
      g[4 * c4 + 0] = (double)g4[c4].x;
      g[4 * c4 + 1] = (double)g4[c4].y;
      g[4 * c4 + 2] = (double)g4[c4].z;
      g[4 * c4 + 3] = (double)g4[c4].w;
    }
#pragma unroll
    for (int c = 0; c < K / 2; ++c) {
      d1[2 * c] = (mk >> (2 * c)) & 1 ? t2[c].x : 0.0;
      d1[2 * c + 1] = (mk >> (2 * c + 1)) & 1 ? t2[c].y : 0.0;
    }
    asm volatile("" : "+v"(o), "+v"(row));
    int j = 0;
    do {
      const int32_t qj = q0 + j;
      const double* __restrict__ Rj = rec + (int64_t)qj * M::R;
      const double* __restrict__ Sj = Rj + 4 + sd * M::SB;
      double s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int c = 0; c < K; ++c) {
        s1 = fma(Sj[c], d1[c], s1);
        s2 = fma(Sj[K + c], g[c], s2);
      }
      const double inv_nj = Rj[0], cqj = Rj[1];
      const int32_t dupj = (int32_t)Sj[2 * K];
      const int64_t* __restrict__ qb = qbase + 4 * (int64_t)qj;
      const int64_t ou = qb[0], oi = qb[1], slot0 = qb[2 + sd];
      const int64_t obj = sd ? oi : ou;
      double infl = (2.0 * e * (s1 + s2) + cqj) * inv_nj;
      if (__builtin_expect(__ballot(o == dupj && lane < len) != 0, 0)) {
        // the test pair's own train row: e = r-hat(u,i) - y, s = x . v (the solve's record)
        if (o == dupj && lane < len) infl = (2.0 * (Rj[3] - (double)y) * Rj[2] + cqj) * inv_nj;
      }
      const int32_t co = (int32_t)(d.out_base - (sd ? qbase[4 * (int64_t)q0 + 1] : qbase[4 * (int64_t)q0]));
      {
        const int64_t ob = obj + co;
        const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<double*>(reinterpret_cast<uintptr_t>(influence) + (uintptr_t)ob * 8), 0, len * n_inf, kBufWord3);
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<int32_t*>(reinterpret_cast<uintptr_t>(rel_idx) + (uintptr_t)ob * 4), 0, len * n_rel, kBufWord3);
        const long long ib = __double_as_longlong(infl);
        __builtin_amdgcn_raw_buffer_store_b64(
            (__attribute__((ext_vector_type(2))) unsigned){(unsigned)(ib & 0xffffffffll), (unsigned)(ib >> 32)}, ri,
            lane * 8, 0, kBufNT);
        __builtin_amdgcn_raw_buffer_store_b32((unsigned)row, rr, lane * 4, 0, kBufNT);
      }
      const int64_t slot = slot0 + co / CH;
      const int32_t pbj = sd ? (int32_t)(oi - ou) : 0;
      if constexpr (KM == 1) {
        double ba = lane < len ? topk_key(infl) : -2.0, bv = infl;
        int bp = lane;
        wave_top1_fast(ba, bp, bv);
        const bool okk = ba > -1.5;
        const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(cand_pos + slot, 0, 4, kBufWord3);
        const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(cand_val + slot, 0, 8, kBufWord3);
        const long long vb = __double_as_longlong(okk ? bv : (double)NAN);
        __builtin_amdgcn_raw_buffer_store_b32((unsigned)(okk ? pbj + co + bp : -1), rp, lane * 4, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64(
            (__attribute__((ext_vector_type(2))) unsigned){(unsigned)(vb & 0xffffffffll), (unsigned)(vb >> 32)}, rv,
            lane * 8, 0, 0);
      } else if constexpr (KM == 2) {
        const bool ok = lane < len;
        const int cp = ok ? pbj + co + lane : -1;
        const double ca = ok ? topk_key(infl) : -2.0;
        double pa = INFINITY;
        int pp = -1;
        for (int t = 0; t < K_top; ++t) {
          double ba = -2.0, bv = 0.0;
          int bp = 0x7fffffff;
          if (cp >= 0 && better(pa, pp, ca, cp) && better(ca, cp, ba, bp)) { ba = ca; bp = cp; bv = infl; }
          wave_best(ba, bp, bv);
          if (lane == 0) {
            const bool okk = ba > -1.5;
            cand_pos[slot * K_top + t] = okk ? bp : -1;
            cand_val[slot * K_top + t] = okk ? bv : NAN;
          }
          pa = ba;
          pp = bp;
        }
      }
    } while (++j < nq);
    if (!more) break;
    ch = nx;
    nx = ch + 1 < cend ? ch + 1 : -1;
    o = no; y = ny; row = nrow; e = ne; mk = nmk;
  }
}

}  // namespace

hipError_t launch_score_mf_runs(int k, int64_t grid, hipStream_t s, const QueryArgs& QA, int64_t Q,
                                const ChunkDesc* cdesc, const int64_t* qbase, const int32_t* slices,
                                const double* rec, int32_t* rel_idx, double* influence, int K, int32_t* cand_pos,
                                double* cand_val, PhaseSpan ps) {
  RunArgs A{};
  for (int sd = 0; sd < 2; ++sd) {
    A.other[sd] = QA.other[sd];
    A.rating[sd] = QA.rating[sd];
    A.row[sd] = QA.row[sd];
    A.emb_other[sd] = QA.t[sd == 0 ? 1 : 0];
    A.bias_other[sd] = QA.t[sd == 0 ? 3 : 2];
  }
#define FIA_RUNS_LAUNCH(KK, KM)                                                                                      \
  hipExtLaunchKernelGGL((k_score_mf_runs<MFm<KK>, KM>), dim3((unsigned)grid), dim3(64), 0, s, ps.a, ps.b, 0, A, Q, \
                        cdesc,                                                                                    \
                     qbase, slices, rec, rel_idx, influence, K, cand_pos, cand_val)
  const int km = K <= 0 ? 0 : K == 1 ? 1 : 2;
  if (k == 16) {
    if (km == 0) FIA_RUNS_LAUNCH(16, 0); else if (km == 1) FIA_RUNS_LAUNCH(16, 1); else FIA_RUNS_LAUNCH(16, 2);
  } else if (k == 8) {
    if (km == 0) FIA_RUNS_LAUNCH(8, 0); else if (km == 1) FIA_RUNS_LAUNCH(8, 1); else FIA_RUNS_LAUNCH(8, 2);
  } else {
    return hipErrorInvalidValue;
  }
#undef FIA_RUNS_LAUNCH
  return hipGetLastError();
}

}  // namespace fia

namespace fia {

hipError_t launch_score_ncf_runs(int k, int64_t grid, hipStream_t s, const QueryArgs& QA, int64_t Q,
                                 const ChunkDesc* cdesc, const int64_t* qbase, const int32_t* slices,
                                 const double* rec, int32_t* rel_idx, double* influence, int K, int32_t* cand_pos,
                                 double* cand_val, PhaseSpan ps) {
  NcfRunArgs A{};
  for (int sd = 0; sd < 2; ++sd) {
    A.other[sd] = QA.other[sd];
    A.rating[sd] = QA.rating[sd];
    A.row[sd] = QA.row[sd];
    A.mask[sd] = reinterpret_cast<const int32_t*>(QA.lgm[sd]);
    A.gmf_other[sd] = QA.t[sd == 0 ? 3 : 2];
  }
  A.resid = QA.lres;
  A.d1tab = QA.d1tab;
  A.N = QA.N;
#define FIA_NRUNS_LAUNCH(KK, KM)                                                                                     \
  hipExtLaunchKernelGGL((k_score_ncf_runs<NCFm<KK>, KM>), dim3((unsigned)grid), dim3(64), 0, s, ps.a, ps.b, 0, A, Q, \
                        cdesc, qbase, slices, rec, rel_idx, influence, K, cand_pos, cand_val)
  const int km = K <= 0 ? 0 : K == 1 ? 1 : 2;
  if (k == 16) {
    if (km == 0) FIA_NRUNS_LAUNCH(16, 0); else if (km == 1) FIA_NRUNS_LAUNCH(16, 1); else FIA_NRUNS_LAUNCH(16, 2);
  } else if (k == 8) {
    if (km == 0) FIA_NRUNS_LAUNCH(8, 0); else if (km == 1) FIA_NRUNS_LAUNCH(8, 1); else FIA_NRUNS_LAUNCH(8, 2);
  } else {
    return hipErrorInvalidValue;
  }
#undef FIA_NRUNS_LAUNCH
  return hipGetLastError();
}

}  // namespace fia

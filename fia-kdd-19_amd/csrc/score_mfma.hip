// MF k in {32, 64}, top-K <= 1: entity-shared scoring on the f64 matrix cores (BASELINE
// config 4, the 20M MF k=64 scoring kernel).  Reference: influence_j = x . grad L(z_j) / n
// for every related rating j of a test rating (src/influence/matrix_factorization.py:237-246).
//
// A work item is <= kMfmaCPI list chunks (256 ratings each) of one entity's list x <= 15 batch
// queries sharing the entity (build_groups).  Per 16-rating tile one 16 x 16 f64 MFMA product
// gives every (rating, query) score, RATINGS AS ROWS and queries as columns:
//   D[j][q] = g_j . x_q + x_bias,q        (q < 15)
//   D[j][15] = g_j . theta_e + c_j = r-hat_j - y_j = e_j
// over K/4 slices of 4 coordinates (slice s pairs coordinate (K/4) kk + s of lane group
// kk = l >> 4, so every lane loads K/4 contiguous coordinates of its rating's gathered row
// and of its query's x) plus one extra slice that adds the per-rating constant
// c_j = (b_e + g + b_o(j)) - y_j into column 15 and the per-query x_bias into the others.
// Lane (kk, n) ends with D[4 r + kk][n] in register r: ratings 4 r + kk of ONE query n, so
// the per-query epilogue state (1/n, c_q, output bases, the running top-1) is one copy per
// lane instead of one per D row; e_j reaches the lanes of row kk by a DPP row broadcast of
// lane 15.  MI355X runs f64 MFMA and f64 VALU on the same units (tools/mb_f64.hip), so the
// epilogue is 2 f64 ops per pair:  influence = fma(e_j * (2/n), D[j][q], c_q / n).
#include "kern.h"

namespace fia {
namespace {

constexpr int kTQB = kMfmaQB;    // queries per work item (column 15 is the entity)
constexpr int kTCPI = kMfmaCPI;  // list chunks per work item

__device__ __forceinline__ double bcast_lane15(double x) {
  // row_newbcast:15 -- every lane of a 16-lane row takes the row's lane 15
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), 0x15F, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x15F, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ long long tkey(double v) {
  // |v|'s bits order like |v| (non-negative doubles); NaN ranks below every number
  const long long b = __double_as_longlong(v) & 0x7fffffffffffffffll;
  return b > 0x7ff0000000000000ll ? -1ll : b;
}

// value of the lane 32 (ROWS2 = true) or 16 (false) apart: v_permlane32/16_swap of x with itself
template <bool ROWS2>
__device__ __forceinline__ unsigned xrows(unsigned x, int lane) {
  if constexpr (ROWS2) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return lane < 32 ? r[1] : r[0];
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return ((lane >> 4) & 1) == 0 ? r[1] : r[0];
  }
}

// the best (key desc, position asc) of the four lanes n, n + 16, n + 32, n + 48
template <bool ROWS2>
__device__ __forceinline__ void best_rows_step(long long& k, int& p, double& v, int lane) {
  const long long vb = __double_as_longlong(v);
  const unsigned klo = xrows<ROWS2>((unsigned)(k & 0xffffffffll), lane), khi = xrows<ROWS2>((unsigned)(k >> 32), lane);
  const unsigned vlo = xrows<ROWS2>((unsigned)(vb & 0xffffffffll), lane), vhi = xrows<ROWS2>((unsigned)(vb >> 32), lane);
  const int p2 = (int)xrows<ROWS2>((unsigned)p, lane);
  const long long k2 = (long long)(((unsigned long long)khi << 32) | klo);
  if (k2 > k || (k2 == k && p2 < p)) {
    k = k2;
    p = p2;
    v = __longlong_as_double((long long)(((unsigned long long)vhi << 32) | vlo));
  }
}

template <class M, bool FULL>
__global__ __launch_bounds__(kScoreThreads) __attribute__((amdgpu_waves_per_eu(3))) void k_score_mf_mfma_t(
    QueryArgs A, int64_t nE, const int64_t* __restrict__ wstart, const int32_t* __restrict__ witems,
    const int64_t* __restrict__ gstart, const int32_t* __restrict__ gq, const int64_t* __restrict__ qbase,
    const double* __restrict__ rec, int32_t* __restrict__ rel_idx, double* __restrict__ influence, int K_top,
    int32_t* __restrict__ cand_pos, double* __restrict__ cand_val, double* __restrict__ sink) {
  static_assert(!M::ncf && (M::K == 32 || M::K == 64), "MF k in {32, 64}");
  constexpr int K = M::K, KS = K / 4, NF4 = KS / 4, TPC = kChunk / 16, CPI = kTCPI, RING = 3;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kk = lane >> 4, cn = lane & 15;
  const int64_t n_items = wstart[nE];
  const int64_t stride = (int64_t)gridDim.x * (kScoreThreads / 64);
  const double gbias = (double)A.t[4][0];
  // every output store is unconditional: lanes without an output (column 15, query columns
  // past the block, positions past the item) write this wave's own sink slots instead.  A
  // store under a lane mask leaves the compiler unsure how many stores follow the next
  // tile's gathers, so it waited with vmcnt(0) -- for the previous tile's stores too
  double* __restrict__ sinkd = sink + ((int64_t)blockIdx.x * (kScoreThreads / 64) + wave) * 128 + lane;
  int32_t* __restrict__ sinki = reinterpret_cast<int32_t*>(sinkd + 64);
  for (int64_t wi = (int64_t)blockIdx.x * (kScoreThreads / 64) + wave; wi < n_items; wi += stride) {
    const int32_t g = witems[3 * wi], cg = witems[3 * wi + 1], qblk = witems[3 * wi + 2];
    const int64_t p0 = (int64_t)cg * (CPI * kChunk);   // first list position of the item
    const int sd = g >= A.U ? 1 : 0;
    const int32_t e = sd ? (int32_t)(g - A.U) : g;
    const int64_t lb = A.ptr[sd][e] + p0;
    const int64_t rem = A.ptr[sd][e + 1] - lb;
    const int len = rem < CPI * kChunk ? (int)rem : CPI * kChunk;
    const int64_t gb = gstart[g] + (int64_t)qblk * kTQB;
    const int64_t gn = gstart[g + 1] - gb;
    const int nq = gn < kTQB ? (int)gn : kTQB;
    const int32_t* __restrict__ oth = A.other[sd] + lb;
    const float* __restrict__ rat = A.rating[sd] + lb;
    const int32_t* __restrict__ rw = A.row[sd] + lb;
    const float* __restrict__ T = sd == 0 ? A.t[1] : A.t[0];     // the other side's table
    const float* __restrict__ bt = sd == 0 ? A.t[3] : A.t[2];
    const float* __restrict__ Es = sd == 0 ? A.t[0] : A.t[1];    // this side's (the entity's) table
    const double bsg = (double)(sd == 0 ? A.t[2] : A.t[3])[e] + gbias;
    // column cn: query cn of the block (cn < nq; columns nq..14 repeat the last query and are
    // never stored) or, cn = 15, the entity itself
    const bool qv = cn < nq;
    const int32_t q = gq[gb + (cn < nq ? cn : nq - 1)];
    const double* __restrict__ R = rec + (int64_t)q * M::R;
    double bq[KS];
    if (cn == 15) {
      const float4* src = reinterpret_cast<const float4*>(Es + (int64_t)e * K + KS * kk);
#pragma unroll
      for (int f = 0; f < NF4; ++f) {
        const float4 t = src[f];
        bq[4 * f] = t.x; bq[4 * f + 1] = t.y; bq[4 * f + 2] = t.z; bq[4 * f + 3] = t.w;
      }
    } else {
      const double2* src = reinterpret_cast<const double2*>(R + 4 + sd * M::SB + K + KS * kk);
#pragma unroll
      for (int f = 0; f < KS / 2; ++f) {
        const double2 t = src[f];
        bq[2 * f] = t.x; bq[2 * f + 1] = t.y;
      }
    }
    const double inv_n = R[0];
    const double al = 2.0 * inv_n, be = R[1] * inv_n;
    const double xb = R[4 + sd * M::SB + 2 * K + 1];
    const int32_t dupo = qv ? (int32_t)R[4 + sd * M::SB + 2 * K + 2] : -1;
    const bool anydup = __ballot(dupo >= 0) != 0;
    int64_t ob, cslot;
    int32_t cpos;
    {
      const longlong2* __restrict__ qb = reinterpret_cast<const longlong2*>(qbase + 4 * (int64_t)q);
      const longlong2 q01 = qb[0], q23 = qb[1];          // {out base user, item}, {slot base user, item}
      ob = (sd ? q01.y : q01.x) + p0;
      cslot = (sd ? q23.y : q23.x) + (int64_t)cg * CPI;
      cpos = (int32_t)(p0 + sd * (q01.y - q01.x));
    }
    // the extra slice's B operand: row 0 = [0 .. 0, 1] (c_j into column 15), row 1 = x_bias
    const double bx = kk == 0 ? (cn == 15 ? 1.0 : 0.0) : (kk == 1 && cn < 15 ? xb : 0.0);
    long long bk = -2;
    int bp = 0x7fffffff;
    double bv = 0.0;
    const int ntl = (len + 15) / 16;
    // software pipeline over the tiles (ring of three): the list entries of tile t + 2 and the
    // gathered rows of tile t + 1 in flight while tile t is scored.  Positions past the item
    // are clamped to its last entry (harmless loads, no branches).
    int32_t so[RING];
    float sy[RING], sbo[RING];
    float4 sb[RING][NF4];
    auto load_list = [&](int t, int k3) {
      const int p = 16 * t + cn < len ? 16 * t + cn : len - 1;
      so[k3] = oth[p];
      sy[k3] = rat[p];
    };
    auto gather = [&](int k3) {
      const float4* row = reinterpret_cast<const float4*>(T + (int64_t)so[k3] * K + KS * kk);
#pragma unroll
      for (int f = 0; f < NF4; ++f) sb[k3][f] = row[f];
      sbo[k3] = bt[so[k3]];
    };
    // per chunk (16 tiles): the best of each query over its four lanes -> the chunk's slot
    auto emit = [&](int chunk) {
      if (K_top <= 0) return;
      long long k1 = bk;
      int p1 = bp;
      double v1 = bv;
      best_rows_step<true>(k1, p1, v1, lane);
      best_rows_step<false>(k1, p1, v1, lane);
      if (kk == 0 && qv) {
        const int64_t slot = (cslot + chunk) * K_top;
        const bool okk = k1 > -2;
        cand_pos[slot] = okk ? (int32_t)(cpos + p1) : -1;
        cand_val[slot] = okk ? v1 : NAN;
      }
      bk = -2; bp = 0x7fffffff; bv = 0.0;
    };
    auto tile = [&](int t, int k3) {
      // this tile's operands pass through an asm with a memory clobber: the loads issued just
      // before (the next tiles' list entries and rows) stay ahead of the wait for these, and
      // the wait counts them (hoisted above them, the wait was vmcnt(0) -- on the loop's
      // first iteration nothing follows the prologue's last gather)
      asm volatile("" : "+v"(sbo[k3]), "+v"(sy[k3]) :: "memory");
#pragma unroll
      for (int f = 0; f < NF4; ++f)
        asm volatile("" : "+v"(sb[k3][f].x), "+v"(sb[k3][f].y), "+v"(sb[k3][f].z), "+v"(sb[k3][f].w));
      // the train rows of this lane's four ratings, needed only by the stores after the
      // MFMA chain (waiting for them there also waits for the next tile's gathers, which
      // the next tile needs at that point anyway)
      int32_t sw[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pw = 16 * t + 4 * r + kk;
        sw[r] = rw[pw < len ? pw : len - 1];
      }
      // the tile's A operands converted first and pinned before the MFMA chain (f64 VALU and
      // f64 MFMA share the DP units: a convert between two MFMAs waits for the first)
      double bd[KS];
#pragma unroll
      for (int f = 0; f < NF4; ++f) {
        bd[4 * f] = sb[k3][f].x; bd[4 * f + 1] = sb[k3][f].y; bd[4 * f + 2] = sb[k3][f].z; bd[4 * f + 3] = sb[k3][f].w;
      }
      // the extra slice's A operand: column 0 = c_j (rating cn), column 1 = 1
      const double cj = (bsg + (double)sbo[k3]) - (double)sy[k3];
      const double ax = kk == 0 ? cj : (kk == 1 ? 1.0 : 0.0);
      if constexpr (KS == 16)
        asm volatile("" : "+v"(bd[0]), "+v"(bd[1]), "+v"(bd[2]), "+v"(bd[3]), "+v"(bd[4]), "+v"(bd[5]),
                     "+v"(bd[6]), "+v"(bd[7]), "+v"(bd[8]), "+v"(bd[9]), "+v"(bd[10]), "+v"(bd[11]),
                     "+v"(bd[12]), "+v"(bd[13]), "+v"(bd[14]), "+v"(bd[15]));
      else
        asm volatile("" : "+v"(bd[0]), "+v"(bd[1]), "+v"(bd[2]), "+v"(bd[3]), "+v"(bd[4]), "+v"(bd[5]),
                     "+v"(bd[6]), "+v"(bd[7]));
      d4_t acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ax, bx, d4_t{0.0, 0.0, 0.0, 0.0}, 0, 0, 0);
#pragma unroll
      for (int sl = 0; sl < KS; ++sl) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(bd[sl], bq[sl], acc, 0, 0, 0);
      double val[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) val[r] = fma(bcast_lane15(acc[r]) * al, acc[r], be);
      if (anydup) {
        // a block query whose test pair is a train row: that row's influence takes e and
        // s = x . v from the record (as the solve wrote them; both copies bit-identical)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * t + 4 * r + kk;
          const int pc = p < len ? p : len - 1;
          if (qv && p < len && oth[pc] == dupo) val[r] = fma((R[3] - (double)rat[pc]) * al, R[2], be);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * t + 4 * r + kk;       // positions ascend with (t, r): strict > keeps the first
        const bool ok = qv && p < len;
        const long long key = ok ? tkey(val[r]) : -2ll;
        const bool take = key > bk;
        bk = take ? key : bk;
        bp = take ? p : bp;
        bv = take ? val[r] : bv;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * t + 4 * r + kk;
        const bool ok = qv && p < len;
        if (FULL || influence) *(ok ? influence + ob + p : sinkd) = val[r];
        if (FULL || rel_idx) *(ok ? rel_idx + ob + p : sinki) = sw[r];
      }
      if (t % TPC == TPC - 1 || t == ntl - 1) emit(t / TPC);
    };
    load_list(0, 0);
    load_list(1, 1);
    gather(0);
    for (int t = 0; t < ntl; t += 3) {
      load_list(t + 2, 2);
      gather(1);
      tile(t, 0);
      if (t + 1 >= ntl) break;
      load_list(t + 3, 0);
      gather(2);
      tile(t + 1, 1);
      if (t + 2 >= ntl) break;
      load_list(t + 4, 1);
      gather(0);
      tile(t + 2, 2);
    }
  }
}

}  // namespace

// sink: 128 doubles per wave of the grid (grid * 4 * 128 * 8 B)
hipError_t launch_score_mf_mfma_t(int k, bool full, int64_t grid, hipStream_t s, const QueryArgs& A, int64_t nE,
                                  const int64_t* wstart, const int32_t* witems, const int64_t* gstart,
                                  const int32_t* gq, const int64_t* qbase, const double* rec, int32_t* rel_idx,
                                  double* influence, int K, int32_t* cand_pos, double* cand_val, double* sink,
                                  PhaseSpan ps) {
#define FIA_T_LAUNCH(KK, F)                                                                                          \
  hipExtLaunchKernelGGL((k_score_mf_mfma_t<MFm<KK>, F>), dim3((unsigned)grid), dim3(kScoreThreads), 0, s, ps.a,  \
                        ps.b, 0, A, nE,                                                                          \
                     wstart, witems, gstart, gq, qbase, rec, rel_idx, influence, K, cand_pos, cand_val, sink)
  if (k == 64) {
    if (full) FIA_T_LAUNCH(64, true); else FIA_T_LAUNCH(64, false);
  } else if (k == 32) {
    if (full) FIA_T_LAUNCH(32, true); else FIA_T_LAUNCH(32, false);
  } else {
    return hipErrorInvalidValue;
  }
#undef FIA_T_LAUNCH
  return hipGetLastError();
}

}  // namespace fia

// MF k in {32, 64}, top-K <= 1: entity-shared scoring on the f64 matrix cores (the config-4
// kernel).  Reference: influence_j = x . grad L(z_j) / n for every related rating j of a test
// rating (u, i) (src/influence/matrix_factorization.py:237-246), x = H_t^-1 v from the solve.
//
// A work item is <= kMfmaCPI chunks of 256 ratings of one entity's list x <= 16 batch queries
// sharing the entity (build_groups).  Per 16-rating tile the scores of every (query, rating)
// pair are one 16x16 tile
//   D = X . G^T      (v_mfma_f64_16x16x4_f64, K/4 slices of 4 coordinates)
// with A rows = the block's 16 queries' x (side block, k coordinates).  The rating's residual
// e_n = r-hat_n - y_n comes from the prepare's list-ordered residuals (k_lres_mf, read with the
// list entries; round 6: row 15 of A was the entity's embedding, D[15][n] the residual's dot --
// 1/16 of the MFMAs and the other side's bias gather per tile).  Slice s pairs coordinate (K/4) kk + s of lane group
// kk = l >> 4: every lane loads K/4 CONTIGUOUS coordinates of its query's x (once per work
// item) and of its rating's gathered row (per tile, 16-B loads).  MI355X runs f64 MFMA and f64
// VALU on the same units (tools/mb_f64.hip: their times add), so the epilogue keeps f64 work
// per pair to 3 ops:
//   influence = fma(e * (2/n), D + x_bias, c_q / n)      (mf:240-246)
// Top-1 candidates: per lane and query a running best over its tiles (|v| bits as an integer
// key), reduced over the 16 lanes of a query row once per chunk.  D layout (f64 16x16x4): lane
// l register r = D[(l >> 4) + 4 r][l & 15]; A[m][k] from lane m + 16 k, B[k][n] from lane
// n + 16 k.
//
// Shared gathers (round 6).  A tile's 16 gathered rows (other-side embeddings, 4 KB at k = 64)
// were a wave's largest cost: rows from row 0 instead of the real ones ran 2.39 vs 3.10 ms per
// config-4 batch, no stores 3.33, no MFMAs 2.73 (same-box ablations) -- the random rows come
// from the Infinity Cache, and the CU's outstanding misses, not bandwidth, bound them.  A
// work item is now (entity chunks) x (a group of kWgBlocks = 4 query blocks of 16): the
// workgroup's four waves score the same tiles, one query block each, and the rows of a tile
// are gathered ONCE per workgroup -- wave h fetches rows 4h .. 4h+3 (one 16-B piece per lane,
// three tiles ahead, into a 3-slot register ring), writes them to a 3-slot LDS ring one tile
// ahead, and one barrier per tile publishes them; each wave reads its B operand from LDS.
// Rows in LDS are XOR-swizzled by 16-B piece (piece u of row r holds source piece u ^ r), so
// the 16 rows of a B-operand read hit 16 different bank groups.  Entity groups with more than
// 16 queries (95 % of the config-4 tiles are item-side, almost all rows live) share
// every gathered row among up to 64 queries: 3.3x fewer row gathers per batch
// (tools/m64_occupancy.py).  The list entries come in blocks of 64 (one per lane, a block
// issued eight tiles before its first tile), broadcast per tile by permlane swaps.
#include <type_traits>

#include "kern.h"

namespace fia {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));   // 16 B in 4 VGPRs

constexpr int kRing = 3;         // staged-row slots (registers: tiles t+1..t+3; LDS: tiles t..t+2)
constexpr int kBlk = 64;         // list entries per block load (one per lane)
constexpr int kBlkTiles = kBlk / 16;
constexpr int kBlkRing = 3;      // block slots: block b + 2 is issued when block b starts
constexpr int kUnroll = 12;      // lcm of the row ring (3) and the block ring in tiles (3 x 4)

// lane 16 R + (l & 15)'s 32-bit value in every lane (R compile-time): two permlane swaps
template <int R>
__device__ __forceinline__ unsigned bcast_row(unsigned x) {
  // permlane32_swap(x, x) -> {[r0 r1 r0 r1], [r2 r3 r2 r3]} (rows of 16 lanes)
  const auto l32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  const unsigned y = R < 2 ? l32[0] : l32[1];
  // permlane16_swap(y, y), y = [a b a b] -> {[a a a a], [b b b b]}
  const auto l16 = __builtin_amdgcn_permlane16_swap(y, y, false, false);
  return (R & 1) ? l16[1] : l16[0];
}
template <int R>
__device__ __forceinline__ double bcast_row_d(double x) {
  const long long b = __double_as_longlong(x);
  const unsigned lo = bcast_row<R>((unsigned)(b & 0xffffffffll)), hi = bcast_row<R>((unsigned)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | lo);
}

template <int CTRL>
__device__ __forceinline__ void ikey_dpp_step(long long& k, int& p, double& v) {
  const long long vb = __double_as_longlong(v);
  const int klo = dpp_i32<CTRL>((int)(k & 0xffffffffll)), khi = dpp_i32<CTRL>((int)(k >> 32));
  const int vlo = dpp_i32<CTRL>((int)(vb & 0xffffffffll)), vhi = dpp_i32<CTRL>((int)(vb >> 32));
  const int p2 = dpp_i32<CTRL>(p);
  const long long k2 = ((long long)khi << 32) | (unsigned)klo;
  if (k2 > k || (k2 == k && p2 < p)) {
    k = k2;
    p = p2;
    v = __longlong_as_double(((long long)vhi << 32) | (unsigned)vlo);
  }
}

__device__ __forceinline__ long long topk_ikey(double v) {
  // |v|'s bits order like |v| (non-negative doubles); NaN ranks below every number
  const long long b = __double_as_longlong(v) & 0x7fffffffffffffffll;
  return b > 0x7ff0000000000000ll ? -1ll : b;
}

template <class M, bool FULL>
__global__ __launch_bounds__(kScoreThreads) __attribute__((amdgpu_waves_per_eu(3))) void k_score_mf_mfma(
    QueryArgs A, int64_t nE, const int64_t* __restrict__ wstart, const int32_t* __restrict__ witems,
    const int64_t* __restrict__ gstart, const int32_t* __restrict__ gq, const int64_t* __restrict__ qbase,
    const double* __restrict__ rec, int32_t* __restrict__ rel_idx, double* __restrict__ influence, int K_top,
    int32_t* __restrict__ cand_pos, double* __restrict__ cand_val) {
  constexpr int CPI = kMfmaCPI;
  static_assert(!M::ncf && (M::K == 32 || M::K == 64), "MF k in {32, 64}");
  static_assert(kScoreThreads == 64 * kWgBlocks, "one wave per query block");
  static_assert(kUnroll % kRing == 0 && kUnroll % 4 == 0 && kUnroll == kBlkRing * kBlkTiles, "ring periods");
  constexpr int K = M::K, KS = K / 4, NF4 = KS / 4, TPC = kChunk / 16;
  constexpr int SG = K / 4;                // 16-B pieces per row
  constexpr int RPW = 64 / SG;             // rows one fetch instruction covers
  constexpr int FW = 16 / RPW;             // waves whose pieces are the tile (k = 64: four; k = 32: two)
  static_assert(FW <= kWgBlocks, "the workgroup covers a tile");
  // the staged rows of three tiles; separate arrays, so the compiler can tell the slots apart.
  // Every wave fetches and stages one 16-B piece per lane (no branch: a load under a branch
  // makes the compiler drain vmcnt), so a slot has 4 x 64 pieces -- at k = 32 the pieces of
  // waves >= FW (rows >= 16: other entries of the block, valid rows) land past the tile's
  // 2 KB and are never read
  constexpr int LSL = 4 * 64 * kWgBlocks;  // floats per slot
  static_assert(LSL >= 16 * K, "a tile fits its slot");
  __shared__ __attribute__((aligned(16))) float lr0[LSL], lr1[LSL], lr2[LSL];
  __shared__ int32_t ccs[kWgBlocks][16][2];     // per query row: candidate slot base, position base
  // each wave's A operand (its 16 queries' x), rows padded by two doubles so
  // the 16 rows of a read fall on 16 bank groups
  constexpr int AST = K + 2;
  __shared__ __attribute__((aligned(16))) double sA[kWgBlocks][16 * AST];
  // per query row of each wave: {2/n, c_q/n, x_bias, {dup other, output run start}} (read per
  // tile; the run start gives the row's aligned output segment and misalignment)
  __shared__ __attribute__((aligned(16))) double sQ[kWgBlocks][16][4];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kk = lane >> 4, cn = lane & 15;     // k-group; A row / B column / D column
  const int64_t n_items = wstart[nE];
  // this lane's staged piece: row fr of the tile, LDS piece lane % SG holds source piece fs
  const int fr = RPW * wave + lane / SG, fs = (lane % SG) ^ (fr % SG);
  for (int64_t wi = blockIdx.x; wi < n_items; wi += gridDim.x) {
    // work item: CPI consecutive chunks (cg) of the entity's list x one group of kWgBlocks
    // query blocks; this wave takes block `wave` of the group
    const int32_t g = witems[3 * wi], cg = witems[3 * wi + 1], qgrp = witems[3 * wi + 2];
    const int64_t p0 = (int64_t)cg * (CPI * kChunk);   // first list position of the item
    const int sd = g >= A.U ? 1 : 0;
    const int32_t e = sd ? (int32_t)(g - A.U) : g;
    const int64_t lb = A.ptr[sd][e] + p0;
    const int64_t rem = A.ptr[sd][e + 1] - lb;
    const int len = rem < CPI * kChunk ? (int)rem : CPI * kChunk;
    const int64_t gb = gstart[g] + (int64_t)qgrp * (kMfmaQB * kWgBlocks) + (int64_t)wave * kMfmaQB;
    const int64_t gn = gstart[g + 1] - gb;
    const int nq = gn <= 0 ? 0 : gn < kMfmaQB ? (int)gn : kMfmaQB;    // wave-uniform; 0: fetch only
    const int32_t* __restrict__ oth = A.other[sd] + lb;
    const float* __restrict__ rat = A.rating[sd] + lb;
    const int32_t* __restrict__ rwp = A.row[sd] + lb;
    const float* __restrict__ T = sd == 0 ? A.t[1] : A.t[0];     // the other side's table
    const double* __restrict__ res = A.lres + (int64_t)sd * A.N + lb;   // e_j by list position
    // list blocks: entry 64 b + lane of the item (clamped to its last entry past the end)
    int32_t lo[kBlkRing], lw[kBlkRing];
    double le[kBlkRing];
    auto load_block = [&](int b, int slot) {
      const int p = kBlk * b + lane < len ? kBlk * b + lane : len - 1;
      lo[slot] = oth[p];
      le[slot] = res[p];
      lw[slot] = rwp[p];
    };
    load_block(0, 0);
    load_block(1, 1);      // (block 2 is the first trip's first step)
    // A operand: lane (row cn, group kk) loads coordinates KS*kk .. KS*kk+KS-1 of its row into
    // this wave's LDS rows (read back per k-slice pair: registers bound the occupancy)
    double a[KS];
    // per D row r (query m = kk + 4 r): influence = fma(e * al, D + xb, be)
    // (32-bit element offsets and candidate slots: a batch holds < 2^29 related ratings and
    // fewer chunks, fia_query_batch; registers are what bounds this kernel's occupancy)
    bool qv[4] = {false, false, false, false};
    if (nq > 0) {
      {
        const int32_t q = gq[gb + (cn < nq ? cn : nq - 1)];
        const double2* src =
            reinterpret_cast<const double2*>(rec + (int64_t)q * M::R + 4 + sd * M::SB + K + KS * kk);
#pragma unroll
        for (int f = 0; f < KS / 2; ++f) {
          const double2 t = src[f];
          a[2 * f] = t.x; a[2 * f + 1] = t.y;
        }
      }
#pragma unroll
      for (int f = 0; f < KS; f += 2)
        *reinterpret_cast<double2*>(&sA[wave][cn * AST + KS * kk + f]) = double2{a[f], a[f + 1]};
      // every query index first, then every per-query load (one wait)
      int32_t qr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = kk + 4 * r;
        qv[r] = m < nq;
        qr[r] = gq[gb + (m < nq ? m : 0)];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double* __restrict__ R = rec + (int64_t)qr[r] * M::R;
        const double inv_n = R[0];
        const int32_t dup_other = (int32_t)R[4 + sd * M::SB + 2 * K + 2];
        const longlong2* __restrict__ qb = reinterpret_cast<const longlong2*>(qbase + 4 * (int64_t)qr[r]);
        const longlong2 q01 = qb[0], q23 = qb[1];          // {out base user, item}, {slot base user, item}
        // the row's output run starts at element ob0 (< 2^29: fia_query_batch's batch bound)
        const uint32_t ob0 = (uint32_t)((sd ? q01.y : q01.x) + p0);
        if (cn == 0) {
          double* __restrict__ w4 = sQ[wave][kk + 4 * r];
          w4[0] = 2.0 * inv_n;
          w4[1] = R[1] * inv_n;
          w4[2] = R[4 + sd * M::SB + 2 * K + 1];
          w4[3] = __longlong_as_double((long long)(((unsigned long long)ob0 << 32) |
                                                    (uint32_t)(qv[r] ? dup_other : -1)));
        }
        // the candidate slot base and position base of the query row, read at each chunk's end
        // (from LDS: registers bound this kernel's occupancy)
        if (cn == 0) {
          ccs[wave][kk + 4 * r][0] = (int32_t)((sd ? q23.y : q23.x) + (int64_t)cg * CPI);
          ccs[wave][kk + 4 * r][1] = (int32_t)(p0 + sd * (q01.y - q01.x));
        }
      }
    }
    // running top-1 per query row: key (|v| bits, -1 NaN, -2 none) and position; the value is
    // the key's bits with the sign kept in bit 31 of the position (positions < 2^30)
    long long bk[4];
    int bp[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { bk[r] = -2; bp[r] = 0x7fffffff; }
    double prv[4] = {0.0, 0.0, 0.0, 0.0};     // previous tile's rotated values (aligned stores)
    int32_t prw[4] = {0, 0, 0, 0};
    const int ntl = (len + 15) / 16;
    // staging: this lane's piece of the rows of tiles t+1 .. t+3 (fetching waves)
    f4v stg[kRing];
    // tile at compile-time position J of the 12-tile period: its block slot and row of 16
    auto fetch = [&](auto jc, auto sc) {
      constexpr int J = decltype(jc)::value, slot = decltype(sc)::value;
      constexpr int BS = (J / kBlkTiles) % kBlkRing, BR = J % kBlkTiles;
      const int32_t of = __shfl((int)lo[BS], (BR * 16 + fr) & 63);
      stg[slot] = *reinterpret_cast<const f4v*>(T + (int64_t)of * K + 4 * fs);
    };
    auto stage = [&](auto sc) {
      constexpr int slot = decltype(sc)::value;
      float* __restrict__ dst = slot == 0 ? lr0 : slot == 1 ? lr1 : lr2;
      *reinterpret_cast<f4v*>(dst + 4 * (64 * wave + lane)) = stg[slot];
    };
    // per chunk (16 tiles): best of each query row over the row's 16 lanes (xor 1..8 stays
    // inside the row) -> the chunk's candidate slot; then the running bests restart
    auto emit = [&](int chunk) {
      if (K_top <= 0) return;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        long long k1 = bk[r];
        int p1 = bp[r] & 0x7fffffff;
        const long long sg = (long long)((unsigned)bp[r] >> 31) << 63;
        double v1 = k1 == -1 ? (double)NAN : __longlong_as_double(k1 | sg);
        // the row's best over its 16 lanes by DPP row rotations (order-independent: strict
        // (key, position) order, unique positions)
        ikey_dpp_step<0x128>(k1, p1, v1);
        ikey_dpp_step<0x124>(k1, p1, v1);
        ikey_dpp_step<0x122>(k1, p1, v1);
        ikey_dpp_step<0x121>(k1, p1, v1);
        if (cn == 0 && qv[r]) {       // (no loads here: a load in the tile loop drains vmcnt)
          const int64_t slot = (int64_t)(ccs[wave][kk + 4 * r][0] + chunk) * K_top;
          const bool okk = k1 > -2;
          cand_pos[slot] = okk ? (int32_t)(ccs[wave][kk + 4 * r][1] + p1) : -1;
          cand_val[slot] = okk ? v1 : NAN;
        }
        bk[r] = -2; bp[r] = 0x7fffffff;
      }
    };
    auto tile = [&](auto jc, int t, auto sc) {
      constexpr int J = decltype(jc)::value, slot = decltype(sc)::value;
      // B operand from the LDS ring: lane (kk, cn) reads row cn, pieces SG/4 kk .. +SG/4-1
      // (swizzled), all converted before the MFMA chain: f64 VALU and f64 MFMA share the
      // MI355X's double-precision units (tools/mb_f64.hip), so a conversion slotted between
      // two MFMAs waits for the first to drain; the empty asm pins them before the chain
      if (nq == 0) return;                       // a fetch-only wave (fewer than 4 blocks)
      const float* __restrict__ src = slot == 0 ? lr0 : slot == 1 ? lr1 : lr2;
      double bd[KS];
#pragma unroll
      for (int f = 0; f < NF4; ++f) {
        const f4v v = *reinterpret_cast<const f4v*>(src + cn * K + 4 * (((NF4 * kk + f) ^ cn) % SG));
        bd[4 * f] = v[0]; bd[4 * f + 1] = v[1]; bd[4 * f + 2] = v[2]; bd[4 * f + 3] = v[3];
      }
      if constexpr (KS == 16)
        asm volatile("" : "+v"(bd[0]), "+v"(bd[1]), "+v"(bd[2]), "+v"(bd[3]), "+v"(bd[4]), "+v"(bd[5]),
                     "+v"(bd[6]), "+v"(bd[7]), "+v"(bd[8]), "+v"(bd[9]), "+v"(bd[10]), "+v"(bd[11]),
                     "+v"(bd[12]), "+v"(bd[13]), "+v"(bd[14]), "+v"(bd[15]));
      else
        asm volatile("" : "+v"(bd[0]), "+v"(bd[1]), "+v"(bd[2]), "+v"(bd[3]), "+v"(bd[4]), "+v"(bd[5]),
                     "+v"(bd[6]), "+v"(bd[7]));
      d4_t acc = {0.0, 0.0, 0.0, 0.0};
      const double* __restrict__ arow = &sA[wave][cn * AST + KS * kk];
#pragma unroll
      for (int sl = 0; sl < KS; sl += 2) {
        const double2 av = *reinterpret_cast<const double2*>(arow + sl);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bd[sl], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bd[sl + 1], acc, 0, 0, 0);
      }
      const int p = 16 * t + cn;                // position in the item of this lane's rating
      const bool pv = p < len;
      constexpr int BS = (J / kBlkTiles) % kBlkRing, BR = J % kBlkTiles;
      const int32_t o = (int32_t)bcast_row<BR>((unsigned)lo[BS]);
      const int32_t w = (int32_t)bcast_row<BR>((unsigned)lw[BS]);
      const double en = bcast_row_d<BR>(le[BS]);                 // e of rating cn
      double al[4], be[4], xb[4];
      int32_t dupo[4], dl[4];
      uint32_t oofs[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double2 ab = *reinterpret_cast<const double2*>(&sQ[wave][kk + 4 * r][0]);
        const double2 xd = *reinterpret_cast<const double2*>(&sQ[wave][kk + 4 * r][2]);
        al[r] = ab.x; be[r] = ab.y; xb[r] = xd.x;
        const unsigned long long pk = (unsigned long long)__double_as_longlong(xd.y);
        dupo[r] = (int32_t)(uint32_t)pk;
        // aligned stores: the row's run starts dl elements into a 16-element (128-B influence,
        // 64-B train-row) segment oofs; lane cn stores segment element cn
        const uint32_t ob0 = (uint32_t)(pk >> 32);
        dl[r] = (int)(ob0 & 15u);
        oofs[r] = ob0 - (uint32_t)dl[r];
      }
      const bool dup = pv && (o == dupo[0] || o == dupo[1] || o == dupo[2] || o == dupo[3]);
      double val[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) val[r] = fma(en * al[r], acc[r] + xb[r], be[r]);
      if (__builtin_expect(__ballot(dup) != 0, 0)) {
        // the test pair's own train row: e = r-hat(u,i) - y, s = x . v (as in k_solve)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (!(pv && qv[r] && o == dupo[r])) continue;
          const int32_t q = gq[gb + kk + 4 * r];
          const double* __restrict__ R = rec + (int64_t)q * M::R;
          const double y = (double)rat[p];
          val[r] = fma((R[3] - y) * al[r], R[2], be[r]);
        }
      }
      // rotate each row by its misalignment dl: lane cn takes element (cn - dl) & 15 -- of
      // this tile (cn >= dl) or, already rotated, of the previous tile (cn < dl) -- so each
      // store is one aligned 16-element segment (whole lines: no line written twice).  All
      // twelve cross-lane reads are issued before the first store: one LDS wait per tile
      // instead of one per row
      double rv[4];
      int32_t rw[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int srcl = ((cn - dl[r]) & 15) + 16 * kk;
        rv[r] = __shfl(val[r], srcl);
        rw[r] = __shfl(w, srcl);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = pv && qv[r];
        const long long key = ok ? topk_ikey(val[r]) : -2ll;
        const bool take = key > bk[r];
        bk[r] = take ? key : bk[r];
        bp[r] = take ? (int)((unsigned)p | ((unsigned)(__double_as_longlong(val[r]) >> 32) & 0x80000000u)) : bp[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool cur = cn >= dl[r];
        const int idx = 16 * t + cn - dl[r];          // element of the run this lane stores
        if (qv[r] && (cur ? idx < len : t > 0)) {
          const uint32_t el = oofs[r] + 16 * t + cn;
          if (FULL || influence) influence[el] = cur ? rv[r] : prv[r];
          if (FULL || rel_idx) rel_idx[el] = cur ? rw[r] : prw[r];
        }
        prv[r] = rv[r];
        prw[r] = rw[r];
      }
      if (t % TPC == TPC - 1 || t == ntl - 1) emit(t / TPC);
    };
    // prologue: the previous item's last tiles are read by every wave before the ring is
    // rewritten; tiles 0..2 fetched, tile 0 staged and published
    __syncthreads();
    fetch(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    fetch(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
    fetch(std::integral_constant<int, 2>{}, std::integral_constant<int, 2>{});
    stage(std::integral_constant<int, 0>{});
    __syncthreads();
    // one trip = kUnroll tiles; step j: block (t + j) / 4 + 2 (when t + j starts a block), the
    // rows of tile t + j + 3 fetched (into the register slot tile t + j's rows left), tile
    // t + j + 1 staged into LDS, one barrier (tile t + j + 1 complete for the next step; every
    // wave is done with tile t + j - 2, whose LDS slot the next step overwrites), then tile
    // t + j from LDS.  Past the item's end the loads are clamped (harmless loads, no branch:
    // a load under a branch drains vmcnt).  ntl is the same in every wave of the workgroup,
    // so every wave takes the same barriers.
    for (int t = 0; t < ntl; t += kUnroll) {
#define FIA_MFMA_STEP(J)                                                                       \
  if constexpr ((J) % kBlkTiles == 0) load_block((t + (J)) / kBlkTiles + 2, ((J) / kBlkTiles + 2) % kBlkRing); \
  fetch(std::integral_constant<int, ((J) + 3) % kUnroll>{}, std::integral_constant<int, (J) % kRing>{});     \
  stage(std::integral_constant<int, ((J) + 1) % kRing>{});                                       \
  __syncthreads();                                                                               \
  tile(std::integral_constant<int, (J)>{}, t + (J), std::integral_constant<int, (J) % kRing>{}); \
  if (t + (J) + 1 >= ntl) break;
      FIA_MFMA_STEP(0)
      FIA_MFMA_STEP(1)
      FIA_MFMA_STEP(2)
      FIA_MFMA_STEP(3)
      FIA_MFMA_STEP(4)
      FIA_MFMA_STEP(5)
      FIA_MFMA_STEP(6)
      FIA_MFMA_STEP(7)
      FIA_MFMA_STEP(8)
      FIA_MFMA_STEP(9)
      FIA_MFMA_STEP(10)
      FIA_MFMA_STEP(11)
#undef FIA_MFMA_STEP
    }
    // the run's tail: the last tile's elements past the last aligned segment
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t ob0 = (uint32_t)((unsigned long long)__double_as_longlong(sQ[wave][kk + 4 * r][3]) >> 32);
      const int dlr = (int)(ob0 & 15u);
      const uint32_t oofr = ob0 - (uint32_t)dlr;
      const int idx = 16 * ntl + cn - dlr;
      if (qv[r] && cn < dlr && idx < len) {
        const uint32_t el = oofr + 16 * ntl + cn;
        if (FULL || influence) influence[el] = prv[r];
        if (FULL || rel_idx) rel_idx[el] = prw[r];
      }
    }
  }
}

}  // namespace

hipError_t launch_score_mf_mfma(int k, bool full, int64_t grid, hipStream_t s, PhaseSpan ps, const QueryArgs& A,
                                int64_t nE, const int64_t* wstart, const int32_t* witems, const int64_t* gstart,
                                const int32_t* gq, const int64_t* qbase, const double* rec, int32_t* rel_idx,
                                double* influence, int K, int32_t* cand_pos, double* cand_val) {
#define FIA_MFMA_LAUNCH(KK, FL)                                                                                     \
  hipExtLaunchKernelGGL((k_score_mf_mfma<MFm<KK>, FL>), dim3((unsigned)grid), dim3(kScoreThreads), 0, s, ps.a, ps.b, \
                        0, A, nE, wstart, witems, gstart, gq, qbase, rec, rel_idx, influence, K, cand_pos, cand_val)
  if (k == 64) {
    if (full) FIA_MFMA_LAUNCH(64, true); else FIA_MFMA_LAUNCH(64, false);
  } else if (k == 32) {
    if (full) FIA_MFMA_LAUNCH(32, true); else FIA_MFMA_LAUNCH(32, false);
  } else {
    return hipErrorInvalidValue;
  }
#undef FIA_MFMA_LAUNCH
  return hipGetLastError();
}

}  // namespace fia

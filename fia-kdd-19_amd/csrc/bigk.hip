// Large-k FIA path: MF k in {128, 256} (side blocks of 129 / 257 coordinates) and
// NCF k in {64, 128, 256} (side blocks of 128 / 256 / 512) -- BASELINE.json config 5
// ("512x512 per-query Hessians, FP64 MFMA Cholesky").  Same math as models.hip
// (mf:164-251, ncf:193-280):
//
//   H_t = (2/n) (A_u (+) B_i) + wd*M + damping*I   (+ coupling iff (u,i) is a train row)
//   x   = H_t^{-1} v,   influence_j = (2 e_j x.g_j + wd x.(M theta)) / n
//
// but every structure is sized for blocks that do not fit a wave's registers or a
// CU's LDS:
//   * per train row, once per prepare: the residual e_j = r-hat_j - y_j and (NCF) the
//     restricted MLP gradient halves g_mlp,side = W1_side . d1_j of both sides
//     (k_resid_mf / k_ncf_rows, the NCF one as four f64-MFMA products per 16 ratings);
//   * per entity: the Gram A_e = sum g g^T in 16x16 tiles (tile-packed lower, fp64),
//     accumulated on v_mfma_f64_16x16x4_f64 from 16-rating slabs staged in LDS
//     (k_big_gram; long lists split into slices, partials summed in slot order);
//   * per (query, side) block -- or per query when the blocks couple -- a blocked
//     left-looking LDL^T (k_big_solve): each 32-column panel is updated from the
//     already-factored columns with MFMA (L streamed from a per-workgroup scratch,
//     D L^T on the fly), factored in LDS, written back.  The right-hand side v rides
//     along as the matrix's extra last row, so its row of L is D^-1 L^-1 v and only the
//     backward solve L^T x = y remains;
//   * scoring over entity chunks shared by every query of the batch with that entity
//     (k_big_score_mfma): the gathered rows / d1_j / e_j are streamed once per chunk
//     into 16 x 16 f64 MFMA products against blocks of 16 query vectors.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "common.h"

namespace fia {
namespace {

typedef double d4_t __attribute__((ext_vector_type(4)));

// C += A B on the f64 matrix cores; lane l supplies A[l&15][l>>4] and B[l>>4][l&15],
// and holds C[(l>>4) + 4r][l&15] in register r.
__device__ __forceinline__ d4_t mfma4(double a, double b, d4_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) void* lds_vp;         // LDS-DMA destination
typedef const __attribute__((address_space(1))) void* glb_vp;   // ... and its global source

__device__ __forceinline__ double wsum(double x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}

// block-wide sum for 256-thread blocks (every thread gets the result)
__device__ __forceinline__ double bsum256(double x, double* red) {
  x = wsum(x);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__device__ __forceinline__ double topk_key(double v) {
  double a = fabs(v);
  return (a != a) ? -1.0 : a;
}
__device__ __forceinline__ bool better(double a1, int p1, double a2, int p2) {
  return a1 > a2 || (a1 == a2 && p1 < p2);
}
__device__ __forceinline__ void wave_best(double& a, int& p, double& v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double oa = __shfl_xor(a, off);
    int op = __shfl_xor(p, off);
    double ov = __shfl_xor(v, off);
    if (better(oa, op, a, p)) { a = oa; p = op; v = ov; }
  }
}

// ------------------------------------------------------------------------------------
// model traits.  A side block has Ds coordinates padded to NPs = 16 T.
//   MF  side [emb (k), bias, 0 pad]  (mf:43-65)    record [x_emb (k), x_bias, dup_other]
//   NCF side [mlp emb (k), gmf emb (k)] (ncf:49-64) record [x_mlp (k), W3g*x_gmf (k), dup_other]
// per-query record: [1/n, c_q, x.v, r-hat(u,i), cq_u, xv_u, cq_i, xv_i, side 0, side 1]
// per-query work:   [n, cdup, esum, r-hat, coupled, -, -, -, v_u, v_i, theta_u, theta_i]
// ------------------------------------------------------------------------------------
template <int K_>
struct BMF {
  static constexpr int K = K_, H = 1, Ds = K + 1, NPs = K + 16, T = NPs / 16;
  static constexpr bool ncf = false;
  static constexpr int SB = K + 2, R = 8 + 2 * SB, QW = 8 + 4 * NPs;
  __host__ __device__ static constexpr bool decayed(int a) { return a < K; }
  // reference theta order [p_u, q_i, b_u, b_i]
  __device__ static int ref_index(int side, int a) { return a < K ? side * K + a : 2 * K + side; }
};

template <int K_>
struct BNCF {
  static constexpr int K = K_, H = K / 2, Ds = 2 * K, NPs = 2 * K, T = NPs / 16;
  static constexpr bool ncf = true;
  static constexpr int SB = 2 * K + 1, R = 8 + 2 * SB, QW = 8 + 4 * NPs;
  __host__ __device__ static constexpr bool decayed(int) { return true; }
  // reference theta order [Pm_u, Qm_i, Pg_u, Qg_i]
  __device__ static int ref_index(int side, int a) { return a < K ? side * K + a : 2 * K + side * K + (a - K); }
};

// Gram tile storage: tile (tr, tc), tc <= tr, in column-major tile order; inside a tile
// element (row m, col n) at m + 16 n.
__host__ __device__ constexpr int tile_off(int T, int tr, int tc) { return tc * T - (tc * (tc - 1)) / 2 + (tr - tc); }
template <class M>
constexpr int64_t gram_words() { return (int64_t)M::T * (M::T + 1) / 2 * 256; }

template <class M>
__device__ __forceinline__ double gram_at(const double* __restrict__ G, int r, int c) {
  const int hi = r > c ? r : c, lo = r > c ? c : r;
  return G[tile_off(M::T, hi >> 4, lo >> 4) * 256 + (hi & 15) + 16 * (lo & 15)];
}

struct BigArgs {
  const int32_t* qu;
  const int32_t* qi;
  int64_t U, I;
  const int64_t* ptr[2];
  const int32_t* row[2];
  const int32_t* other[2];
  const float* rating[2];
  const double* gram[2];
  const double* l1[2];
  const double* resid;
  const double* gm[2];     // NCF g_mlp per side, by train row
  const int32_t* slot[2];  // Gram cache slot per entity (nullptr = identity)
  const float* t[10];
  double wd, damping;
  PairTable pairs;
};

// ------------------------------------------------------------------------------------
// entities referenced by a query set (fia_prepare_for)
__global__ void k_mark(int64_t Q, const int32_t* __restrict__ qu, const int32_t* __restrict__ qi, int64_t U,
                       int64_t I, uint8_t* __restrict__ mark) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < Q; q += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = qu[q], i = qi[q];
    if (u >= 0 && u < U && i >= 0 && i < I) {
      mark[u] = 1;
      mark[U + i] = 1;
    }
  }
}

__global__ void k_check_cover(int64_t Q, const int32_t* __restrict__ qu, const int32_t* __restrict__ qi, int64_t U,
                              int64_t I, const int32_t* __restrict__ slot0, const int32_t* __restrict__ slot1,
                              int32_t* __restrict__ flag) {
  int bad = 0;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < Q; q += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = qu[q], i = qi[q];
    if (u >= 0 && u < U && i >= 0 && i < I) bad |= slot0[u] < 0 || slot1[i] < 0;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// per-position entity of a side's lists: self[p] = e with ptr[e] <= p < ptr[e+1]
// ------------------------------------------------------------------------------------
__global__ void k_self(int64_t N, int64_t n_ent, const int64_t* __restrict__ ptr, int32_t* __restrict__ self) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = n_ent;
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (ptr[mid] <= p) lo = mid; else hi = mid - 1;
    }
    self[p] = (int32_t)lo;
  }
}

// MF residual by train row (user-major pass): e_j = p_u.q_i + b_u + b_i + g - y_j (mf:89-116).
// fia_prepare_for (mark != nullptr): only the rows the shard's scoring reads -- those in a
// cached user's or a cached item's list (a query (u, i) scores exactly the lists of u and i)
template <int K>
__global__ void k_resid_mf(int64_t N, const int32_t* __restrict__ self0, const int32_t* __restrict__ other0,
                           const int32_t* __restrict__ row0, const float* __restrict__ rat0,
                           const float* __restrict__ P, const float* __restrict__ Qt, const float* __restrict__ bu,
                           const float* __restrict__ bi, const float* __restrict__ gb, double* __restrict__ resid,
                           const uint8_t* __restrict__ mark, int64_t U) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = self0[p], i = other0[p];
    if (mark && !mark[u] && !mark[U + i]) continue;
    const float4* a = reinterpret_cast<const float4*>(P + (int64_t)u * K);
    const float4* b = reinterpret_cast<const float4*>(Qt + (int64_t)i * K);
    double acc = 0.0;
#pragma unroll 8
    for (int c = 0; c < K / 4; ++c) {
      const float4 x = a[c], y = b[c];
      acc = fma((double)x.x, (double)y.x, acc);
      acc = fma((double)x.y, (double)y.y, acc);
      acc = fma((double)x.z, (double)y.z, acc);
      acc = fma((double)x.w, (double)y.w, acc);
    }
    resid[row0[p]] = acc + (double)bu[u] + (double)bi[i] + (double)gb[0] - (double)rat0[p];
  }
}

// NCF layer-1 halves L1[e] = emb_e . W1[row_off : row_off + k]  (fp64)
template <int K>
__global__ void k_l1_big(const float* __restrict__ emb, const float* __restrict__ W1, int row_off, int64_t n_ent,
                         double* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_ent * K;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / K;
    const int c = (int)(t % K);
    const float* x = emb + e * K;
    double acc = 0.0;
    for (int a = 0; a < K; ++a) acc = fma((double)x[a], (double)W1[(int64_t)(row_off + a) * K + c], acc);
    out[t] = acc;
  }
}

// NCF per train row (one 4-wave workgroup per 16 list positions of side `pass`; the
// waves split each product's output tiles), all products on the f64 matrix cores
// (ncf:102-145, TF ReluGrad masks):
//   z1 = L1u + L1i + b1,  z2 = relu(z1) W2 + b2,  d2 = 1[z2>0] W3m,
//   d1 = 1[z1>0] (W2 d2),  r-hat = W3m.relu(z2) + W3g.(Pg_u*Qg_i) + b3
// pass < 0 (full prepare): user-major positions, g_mlp of both sides for every row.
// pass = sd (fia_prepare_for): side sd's positions, tiles without a cached entity's row
// skipped, g_mlp of side sd only -- a cached entity's list is one contiguous run of its
// side's positions, so the work is dense.  A row in both kinds of list gets its
// residual from both passes: the same arithmetic, the same bits.
constexpr int kRowWaves = 4;

// The MLP weights as f64 MFMA B-operand fragments, built once per prepare (3 k^2 doubles,
// L2-resident): fragment (t, p) of a product is 64 lanes x 2 doubles, lane (ml, kl)
// holding the weights of output column 16t + ml at reduction indices 8p + 2kl + {0, 1}
// (the A operand reads the same two indices as one 16-B LDS word), so every B load of
// k_ncf_rows is one contiguous 1-KB dwordx4 wave load covering two MFMAs instead of
// sixteen scattered 16-B row pieces and a convert per MFMA.
//   [0, HK)        z2 = relu(z1) W2:  W2[kidx][col]      t < H/16, p < K/8
//   [HK, 2HK)      W2 d2:             W2[col][kidx]      t < K/16, p < H/8
//   [2HK, 2HK+2K^2) g_mlp, side sd:   W1[sd K + col][kidx] t < K/16, p < K/8
template <int K>
__global__ void k_ncf_wfrag(const float* __restrict__ W1, const float* __restrict__ W2, double* __restrict__ wf) {
  constexpr int H = K / 2;
  constexpr int64_t n = (int64_t)3 * K * K;
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n; f += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(f & 1), lane = (int)((f >> 1) & 63);
    const int64_t tp = f >> 7;   // fragment index (t, p) within its product
    const int ml = lane & 15, kl = lane >> 4;
    double x;
    if (f < (int64_t)H * K) {
      const int t = (int)(tp / (K / 8)), p = (int)(tp % (K / 8));
      x = W2[(8 * p + 2 * kl + i) * H + 16 * t + ml];
    } else if (f < (int64_t)2 * H * K) {
      const int64_t q = tp - (int64_t)H * K / 128;
      const int t = (int)(q / (H / 8)), p = (int)(q % (H / 8));
      x = W2[(16 * t + ml) * H + 8 * p + 2 * kl + i];
    } else {
      const int64_t q = tp - (int64_t)2 * H * K / 128;
      const int sd = (int)(q / (K / 16 * (K / 8)));
      const int64_t r = q % (K / 16 * (K / 8));
      const int t = (int)(r / (K / 8)), p = (int)(r % (K / 8));
      x = W1[(int64_t)(sd * K + 16 * t + ml) * K + 8 * p + 2 * kl + i];
    }
    wf[f] = x;
  }
}

template <int K>
__global__ __launch_bounds__(64 * kRowWaves) void k_ncf_rows(
    int64_t N, int pass, const int32_t* __restrict__ self0, const int32_t* __restrict__ other0,
    const int32_t* __restrict__ row0, const float* __restrict__ rat0, const double* __restrict__ l1u,
    const double* __restrict__ l1i, const float* __restrict__ b1, const float* __restrict__ W2,
    const float* __restrict__ b2, const float* __restrict__ W3, const float* __restrict__ b3,
    const float* __restrict__ Pg, const float* __restrict__ Qg, const double2* __restrict__ wf,
    double* __restrict__ gm0, double* __restrict__ gm1, double* __restrict__ resid,
    const uint8_t* __restrict__ mark, int64_t U) {
  constexpr int H = K / 2, LZ = K + 4, LD2 = H + 4, NW = kRowWaves;
  __shared__ __attribute__((aligned(16))) double Z1[16 * LZ];
  __shared__ __attribute__((aligned(16))) double D2[16 * LD2];
  const double2* __restrict__ Fz2 = wf;
  const double2* __restrict__ Fd1 = wf + H * K / 2;
  const double2* __restrict__ Fg = wf + H * K;
  __shared__ double part_mlp[NW][16];
  __shared__ double part_gmf[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ml = lane & 15, kl = lane >> 4;
  for (int64_t tile = blockIdx.x; tile * 16 < N; tile += gridDim.x) {
    const int64_t p0 = tile * 16;
    const int64_t my = p0 + ml;
    const bool v = my < N;
    const int32_t s_l = v ? self0[my] : 0, o_l = v ? other0[my] : 0, j_l = v ? row0[my] : 0;
    const int32_t u_l = pass == 1 ? o_l : s_l, i_l = pass == 1 ? s_l : o_l;
    // fia_prepare_for: g_mlp of a side is needed only for rows in a cached entity's list
    const bool need_u = v && pass != 1 && (!mark || mark[u_l]);
    const bool need_i = v && pass != 0 && (!mark || mark[U + i_l]);
    const bool any_u = __any(need_u), any_i = __any(need_i);
    if (pass >= 0 && !(any_u || any_i)) continue;   // uniform over the workgroup (same tile)
    __syncthreads();
    for (int e = tid; e < 16 * K; e += 64 * NW) {
      const int r = e / K, c = e % K;
      const int32_t u = __shfl(u_l, r), i = __shfl(i_l, r);
      Z1[r * LZ + c] = l1u[(int64_t)u * K + c] + l1i[(int64_t)i * K + c] + (double)b1[c];
    }
    __syncthreads();
    double mlp[4] = {0.0, 0.0, 0.0, 0.0};
    for (int t = w; t < H / 16; t += NW) {
      d4_t acc = {0.0, 0.0, 0.0, 0.0};
      const double2* __restrict__ fb = Fz2 + t * (K / 8) * 64 + lane;
#pragma unroll 4
      for (int p = 0; p < K / 8; ++p) {
        const double2 z = *reinterpret_cast<const double2*>(Z1 + ml * LZ + 8 * p + 2 * kl);
        const double2 b = fb[64 * p];
        acc = mfma4(z.x > 0.0 ? z.x : 0.0, b.x, acc);
        acc = mfma4(z.y > 0.0 ? z.y : 0.0, b.y, acc);
      }
      const int d = 16 * t + ml;
      const double w3m = (double)W3[d], bb = (double)b2[d];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double z2 = acc[r] + bb;
        const bool on = z2 > 0.0;
        mlp[r] += on ? w3m * z2 : 0.0;
        D2[(kl + 4 * r) * LD2 + d] = on ? w3m : 0.0;
      }
    }
    // this wave's MLP partial of row kl + 4r sits in lane 16 kl after the reduction
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double m = mlp[r];
      m += __shfl_xor(m, 1);
      m += __shfl_xor(m, 2);
      m += __shfl_xor(m, 4);
      m += __shfl_xor(m, 8);
      if (ml == 0) part_mlp[w][kl + 4 * r] = m;
    }
    // gmf dot of rows w, w + NW, ... (wave-wide over the k coordinates)
    for (int r = w; r < 16; r += NW) {
      const int32_t u = __shfl(u_l, r), i = __shfl(i_l, r);
      double part = 0.0;
      for (int c = lane; c < K; c += 64)
        part = fma((double)W3[H + c] * (double)Pg[(int64_t)u * K + c], (double)Qg[(int64_t)i * K + c], part);
      part = wsum(part);
      if (lane == 0) part_gmf[r] = part;
    }
    __syncthreads();
    for (int t = w; t < K / 16; t += NW) {
      d4_t acc = {0.0, 0.0, 0.0, 0.0};
      const double2* __restrict__ fb = Fd1 + t * (H / 8) * 64 + lane;
#pragma unroll 4
      for (int p = 0; p < H / 8; ++p) {
        const double2 a = *reinterpret_cast<const double2*>(D2 + ml * LD2 + 8 * p + 2 * kl);
        const double2 b = fb[64 * p];
        acc = mfma4(a.x, b.x, acc);
        acc = mfma4(a.y, b.y, acc);
      }
      const int c = 16 * t + ml;
#pragma unroll
      for (int r = 0; r < 4; ++r) {           // Z1 becomes D1 (each lane rewrites what it read)
        double* z = Z1 + (kl + 4 * r) * LZ + c;
        *z = *z > 0.0 ? acc[r] : 0.0;
      }
    }
    __syncthreads();
    // g_mlp of both sides: D1 . W1_side^T (W1 rows [0, k) act on Pm, rows [k, 2k) on Qm)
#pragma unroll 1
    for (int sd = 0; sd < 2; ++sd) {
      if (!(sd ? any_i : any_u)) continue;
      double* __restrict__ gm = sd ? gm1 : gm0;
      for (int t = w; t < K / 16; t += NW) {
        d4_t acc = {0.0, 0.0, 0.0, 0.0};
        const double2* __restrict__ fb = Fg + (sd * (K / 16) + t) * (K / 8) * 64 + lane;
#pragma unroll 4
        for (int p = 0; p < K / 8; ++p) {
          const double2 a = *reinterpret_cast<const double2*>(Z1 + ml * LZ + 8 * p + 2 * kl);
          const double2 b = fb[64 * p];
          acc = mfma4(a.x, b.x, acc);
          acc = mfma4(a.y, b.y, acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = kl + 4 * r;
          const int32_t j = __shfl(j_l, row);
          if (p0 + row < N) gm[(int64_t)j * K + 16 * t + ml] = acc[r];
        }
      }
    }
    if (w == 0 && lane < 16 && v) {
      double m = 0.0;
#pragma unroll
      for (int q = 0; q < NW; ++q) m += part_mlp[q][lane];
      resid[j_l] = m + part_gmf[lane] + (double)b3[0] - (double)rat0[my];
    }
  }
}

// ------------------------------------------------------------------------------------
// Entity Gram caches on the f64 matrix cores.  A workgroup (8 waves) takes one slice
// (<= kBigSlice ratings) of one entity's list and one group of output tiles; per
// 16 ratings it stages the g rows in LDS (MF: the gathered other-side embedding + 1;
// NCF: W1_side . d1_j by MFMA + W3g * gmf_other) and every wave adds the rank-16
// update of its tiles (4 MFMAs per tile).
// ------------------------------------------------------------------------------------
constexpr int kGW = 8;              // waves per Gram workgroup
constexpr int kBigSlice = 2048;     // ratings per Gram work item

template <class M>
struct GramCfg {
  static constexpr int NTL = M::T * (M::T + 1) / 2;
  // accumulator tiles per wave (NCF: fewer, for the prefetched slab registers)
  static constexpr int MAXPER = M::ncf ? 14 : 18;
  static constexpr int NG = (NTL + kGW * MAXPER - 1) / (kGW * MAXPER);  // tile groups (workgroups per slice)
  static constexpr int TPG = (NTL + NG - 1) / NG;
  static constexpr int PER = (TPG + kGW - 1) / kGW;
  static constexpr int LDT = 18;            // NCF slab: coordinate-major, 16 ratings + 2 pad
  static constexpr int LDG = M::NPs + 16;   // MF slab: rating-major row stride (doubles)
  static constexpr int SLAB = M::ncf ? M::NPs * LDT : 16 * LDG;
};

// One staging thread's share of a 16-rating slab, loaded into registers one slab ahead and
// written to LDS as f64.  MF: the gathered other-side embedding, then the constant 1 of
// the bias coordinate, rating-major; NCF: g_mlp,j of the side (precomputed by k_ncf_rows),
// then W3g * gmf_other, coordinate-major (slab[coord * LDT + rating]: a lane's two ratings
// of an MFMA pair are one 16-B read, and the 16 lanes of a coordinate write 32 consecutive
// dwords; config-5 NCF prepare 114.7 -> 107.1 ms, same-box A/B; at MF k = 256 it measured
// 20.1 vs 19.4 ms and MF keeps the rating-major slab)
template <class M, bool NCF = M::ncf>
struct GramStage;

template <class M>
struct GramStage<M, false> {   // rating-major: row r of the slab, coordinates pp * PERT + [0, PERT)
  static constexpr int K = M::K, PERT = K / 32, LDG = GramCfg<M>::LDG;
  float4 x[PERT / 4];
  bool valid;
  __device__ void fetch(const int32_t* __restrict__ other, const int32_t*, const float* __restrict__ emb,
                        const double*, int64_t pos, int r, int rem, int pp) {
    valid = r < rem;
    const int32_t o = valid ? other[pos + r] : 0;
    const float4* src = reinterpret_cast<const float4*>(emb + (int64_t)o * K + pp * PERT);
#pragma unroll
    for (int c = 0; c < PERT / 4; ++c) x[c] = src[c];
  }
  __device__ void put(double* __restrict__ G, const double*, int r, int pp) const {
    double* row = G + r * LDG;
#pragma unroll
    for (int c = 0; c < PERT / 4; ++c) {
      double* d = row + pp * PERT + 4 * c;
      d[0] = valid ? (double)x[c].x : 0.0;
      d[1] = valid ? (double)x[c].y : 0.0;
      d[2] = valid ? (double)x[c].z : 0.0;
      d[3] = valid ? (double)x[c].w : 0.0;
    }
    if (pp < 16) row[K + pp] = (pp == 0 && valid) ? 1.0 : 0.0;
  }
};

template <class M>
struct GramStage<M, true> {
  static constexpr int K = M::K, PERT = K / 32, LDT = GramCfg<M>::LDT;
  double m[PERT];
  float g[PERT];
  bool valid;
  __device__ void fetch(const int32_t* __restrict__ other, const int32_t* __restrict__ rowid,
                        const float* __restrict__ emb, const double* __restrict__ gms, int64_t pos, int r, int rem,
                        int q) {
    valid = r < rem;
    const int32_t o = valid ? other[pos + r] : 0;
    const int32_t j = valid ? rowid[pos + r] : 0;
    const double* msrc = gms + (int64_t)j * K + q * PERT;
    const float* gsrc = emb + (int64_t)o * K + q * PERT;
#pragma unroll
    for (int c = 0; c < PERT; ++c) {
      m[c] = msrc[c];
      g[c] = gsrc[c];
    }
  }
  __device__ void put(double* __restrict__ G, const double* __restrict__ w3g, int r, int q) const {
    double* d = G + q * PERT * LDT + r;
#pragma unroll
    for (int c = 0; c < PERT; ++c) {
      d[c * LDT] = valid ? m[c] : 0.0;
      d[(K + c) * LDT] = valid ? w3g[q * PERT + c] * (double)g[c] : 0.0;
    }
  }
};

template <class M>
__global__ __launch_bounds__(64 * kGW) void k_big_gram(int sd, int64_t n_items, const int32_t* __restrict__ items,
                                                       const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ other,
                                                       const int32_t* __restrict__ rowid,
                                                       const float* __restrict__ emb_other,
                                                       const double* __restrict__ gms, const float* __restrict__ W3,
                                                       double* __restrict__ gram, double* __restrict__ part) {
  using C = GramCfg<M>;
  constexpr int T = M::T, LDT = C::LDT, LDG = C::LDG, PER = C::PER;
  constexpr int64_t GW = gram_words<M>();
  // two slab buffers: slab n is written to Gs[n & 1] while the waves may still read slab
  // n - 1 from the other one, so one barrier per slab, and the next slab's global loads
  // are issued before this slab's MFMAs (they land while the matrix cores run)
  __shared__ __attribute__((aligned(16))) double Gs[2][C::SLAB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ml = lane & 15, kl = lane >> 4;
  // NG > 2 (NCF k = 256): XCD-aware order -- block b runs on XCD b % 8 and the NG tile
  // groups of one slice are blocks 8 apart (same XCD, dispatched together), so a slab's
  // gathered rows come from HBM once per slice instead of once per group; gridDim.x is a
  // multiple of 8 NG, so a block keeps its group (config-5 NCF prepare 117.0 -> 115.3 ms;
  // at NG = 2, MF k = 256, the plain 2-D grid measured faster: 19.5 vs 20.4 ms)
  constexpr bool XG = C::NG > 2;
  const int grp = XG ? (int)((blockIdx.x >> 3) % C::NG) : (int)blockIdx.y;
  const int64_t n_vb = XG ? ((n_items + 7) / 8) * 8 * C::NG : n_items;
  // staging thread: rating r, coordinate chunk q (NCF: 16 lanes per coordinate; MF: 32
  // threads per rating row)
  const int r = M::ncf ? tid & 15 : tid >> 5, q = M::ncf ? tid >> 4 : tid & 31;
  __shared__ double w3g[M::ncf ? M::K : 1];   // NCF: W3's GMF weights (f64) for the staging
  if constexpr (M::ncf)
    for (int c = tid; c < M::K; c += 64 * kGW) w3g[c] = (double)W3[M::H + c];
  __syncthreads();
  GramStage<M> stage;
  const int tend = (grp + 1) * C::TPG < C::NTL ? (grp + 1) * C::TPG : C::NTL;
  int tr_[PER], tc_[PER];
  bool on_[PER];
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int idx = grp * C::TPG + wave * PER + p;
    on_[p] = idx < tend;
    int tr = 0;
    while ((tr + 1) * (tr + 2) / 2 <= idx) ++tr;
    tr_[p] = on_[p] ? tr : 0;
    tc_[p] = on_[p] ? idx - tr * (tr + 1) / 2 : 0;
  }
  // a slot past the group's last tile (on_ false) computes tile (0, 0) and is not stored:
  // a few % more MFMAs instead of a scalar branch in front of every one
  int buf = 0;
  for (int64_t vb = blockIdx.x; vb < n_vb; vb += gridDim.x) {
    const int64_t it = XG ? 8 * (vb / (8 * C::NG)) + (vb & 7) : vb;
    if (it >= n_items) continue;   // uniform over the block
    const int32_t e = items[4 * it], start = items[4 * it + 1], len = items[4 * it + 2], dst = items[4 * it + 3];
    const int64_t lb = ptr[e] + start;
    d4_t acc[PER];
#pragma unroll
    for (int p = 0; p < PER; ++p) acc[p] = d4_t{0.0, 0.0, 0.0, 0.0};
    stage.fetch(other, rowid, emb_other, gms, lb, r, len, q);
    for (int t0 = 0; t0 < len; t0 += 16, buf ^= 1) {
      double* __restrict__ G = Gs[buf];
      stage.put(G, w3g, r, q);
      __syncthreads();
      if (t0 + 16 < len) stage.fetch(other, rowid, emb_other, gms, lb + t0 + 16, r, len - t0 - 16, q);
      // MFMA pair h: lane (m, g) supplies ratings 8h + 2g and 8h + 2g + 1 of coordinate
      // 16 tr + m (A) / 16 tc + m (B), one 16-B read each
      if constexpr (M::ncf) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const double* gc = G + ml * LDT + 8 * h + 2 * kl;
#pragma unroll
          for (int p = 0; p < PER; ++p) {
            const double2 a = *reinterpret_cast<const double2*>(gc + 16 * LDT * tr_[p]);
            const double2 b = *reinterpret_cast<const double2*>(gc + 16 * LDT * tc_[p]);
            acc[p] = mfma4(a.x, b.x, acc[p]);
            acc[p] = mfma4(a.y, b.y, acc[p]);
          }
        }
      } else {
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const double* gr = G + (4 * s4 + kl) * LDG + ml;
#pragma unroll
          for (int p = 0; p < PER; ++p) acc[p] = mfma4(gr[16 * tr_[p]], gr[16 * tc_[p]], acc[p]);
        }
      }
    }
    double* out = dst >= 0 ? gram + (int64_t)dst * GW : part + (int64_t)(-dst - 1) * GW;
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      if (!on_[p]) continue;
      double* tb = out + (int64_t)tile_off(T, tr_[p], tc_[p]) * 256 + 16 * ml;
#pragma unroll
      for (int r = 0; r < 4; ++r) tb[kl + 4 * r] = acc[p][r];
    }
  }
}

// partial Grams of a long list summed in slot order; blockIdx.y splits the GW words so a
// handful of long lists still spreads over every CU
constexpr int kCombSplit = 64;
__global__ void k_big_combine(int64_t n_comb, const int32_t* __restrict__ comb, int64_t GW,
                              const double* __restrict__ part, double* __restrict__ gram) {
  const int64_t per = (GW + kCombSplit - 1) / kCombSplit;
  const int64_t t0 = (int64_t)blockIdx.y * per, t1 = t0 + per < GW ? t0 + per : GW;
  for (int64_t w = blockIdx.x; w < n_comb; w += gridDim.x) {
    const int32_t gs = comb[4 * w], first = comb[4 * w + 1], ns = comb[4 * w + 2];
    const double* __restrict__ src = part + (int64_t)first * GW;
    for (int64_t t = t0 + threadIdx.x; t < t1; t += blockDim.x) {
      double s = 0.0;
      for (int k = 0; k < ns; ++k) s += src[(int64_t)k * GW + t];
      gram[(int64_t)gs * GW + t] = s;
    }
  }
}

// ------------------------------------------------------------------------------------
// Per-query prologue (one 256-thread block per query): n, the pair terms, r-hat(u,i),
// theta_t and v = d r-hat(u,i) / d theta_t (gnn:155, mf:194,201 / ncf:222,229); append
// the query's systems to the solve lists.
// ------------------------------------------------------------------------------------
template <class M>
__global__ __launch_bounds__(256) void k_big_prologue(BigArgs A, int64_t Q, double* __restrict__ qwork,
                                                      int32_t* __restrict__ syslist, int32_t* __restrict__ cpllist) {
  constexpr int K = M::K, NPs = M::NPs;
  __shared__ double red[4];
  __shared__ double z1[M::ncf ? K : 1], d2[M::ncf ? M::H : 1], d1[M::ncf ? K : 1];
  const int tid = threadIdx.x;
  for (int64_t q = blockIdx.x; q < Q; q += gridDim.x) {
    const int32_t u = A.qu[q], i = A.qi[q];
    double* qw = qwork + q * M::QW;
    bool ok = u >= 0 && u < A.U && i >= 0 && i < A.I;
    if (ok && A.slot[0]) ok = A.slot[0][u] >= 0 && A.slot[1][i] >= 0;   // not cached: NaN (checked by the ABI)
    const int64_t n = ok ? (A.ptr[0][u + 1] - A.ptr[0][u]) + (A.ptr[1][i + 1] - A.ptr[1][i]) : 0;
    if (n == 0) {
      if (tid == 0) qw[0] = 0.0;
      continue;
    }
    double* vu = qw + 8;
    double* vi = vu + NPs;
    double* thu = vi + NPs;
    double* thi = thu + NPs;
    double rhat;
    if constexpr (!M::ncf) {
      const float* P = A.t[0] + (int64_t)u * K;
      const float* Qt = A.t[1] + (int64_t)i * K;
      double part = 0.0;
      for (int a = tid; a < NPs; a += 256) {
        const double pu = a < K ? (double)P[a] : 0.0, qi = a < K ? (double)Qt[a] : 0.0;
        part = fma(pu, qi, part);
        vu[a] = a < K ? qi : (a == K ? 1.0 : 0.0);
        vi[a] = a < K ? pu : (a == K ? 1.0 : 0.0);
        thu[a] = a < K ? pu : (a == K ? (double)A.t[2][u] : 0.0);
        thi[a] = a < K ? qi : (a == K ? (double)A.t[3][i] : 0.0);
      }
      rhat = bsum256(part, red) + (double)A.t[2][u] + (double)A.t[3][i] + (double)A.t[4][0];
    } else {
      constexpr int H = M::H;
      const float* W1 = A.t[4];
      const float* W2 = A.t[6];
      const float* W3 = A.t[8];
      __syncthreads();
      for (int c = tid; c < K; c += 256)
        z1[c] = A.l1[0][(int64_t)u * K + c] + A.l1[1][(int64_t)i * K + c] + (double)A.t[5][c];
      __syncthreads();
      double mlp = 0.0;
      for (int d = tid; d < H; d += 256) {
        double z2 = (double)A.t[7][d];
        for (int c = 0; c < K; ++c) z2 = fma((double)W2[c * H + d], z1[c] > 0.0 ? z1[c] : 0.0, z2);
        const bool on = z2 > 0.0;
        mlp += on ? (double)W3[d] * z2 : 0.0;
        d2[d] = on ? (double)W3[d] : 0.0;
      }
      __syncthreads();
      for (int c = tid; c < K; c += 256) {
        double t = 0.0;
        for (int d = 0; d < H; ++d) t = fma((double)W2[c * H + d], d2[d], t);
        d1[c] = z1[c] > 0.0 ? t : 0.0;
      }
      __syncthreads();
      double gmf = 0.0;
      for (int a = tid; a < K; a += 256) {
        double su = 0.0, si = 0.0;
        for (int c = 0; c < K; ++c) {
          su = fma((double)W1[(int64_t)a * K + c], d1[c], su);
          si = fma((double)W1[(int64_t)(K + a) * K + c], d1[c], si);
        }
        const double pm = A.t[0][(int64_t)u * K + a], qm = A.t[1][(int64_t)i * K + a];
        const double pg = A.t[2][(int64_t)u * K + a], qg = A.t[3][(int64_t)i * K + a];
        const double w3g = (double)W3[H + a];
        vu[a] = su;
        vi[a] = si;
        vu[K + a] = w3g * qg;        // d r / d Pg_u = W3g * Qg_i
        vi[K + a] = w3g * pg;        // d r / d Qg_i = W3g * Pg_u
        thu[a] = pm;
        thu[K + a] = pg;
        thi[a] = qm;
        thi[K + a] = qg;
        gmf = fma(w3g * pg, qg, gmf);
      }
      rhat = bsum256(mlp + gmf, red) + (double)A.t[9][0];
    }
    if (tid == 0) {
      double cdup, rsum;
      A.pairs.lookup((unsigned long long)u * (unsigned long long)A.I + (unsigned long long)i, cdup, rsum);
      qw[0] = (double)n;
      qw[1] = cdup;
      qw[2] = cdup * rhat - rsum;
      qw[3] = rhat;
      qw[4] = cdup > 0.0 ? 1.0 : 0.0;
      if (cdup > 0.0) {
        const int s = atomicAdd(cpllist, 1);
        cpllist[1 + s] = (int32_t)q;
      } else {
        const int s = atomicAdd(syslist, 2);
        syslist[1 + s] = (int32_t)(2 * q);
        syslist[2 + s] = (int32_t)(2 * q + 1);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Blocked left-looking LDL^T + solve, one 512-thread workgroup per system (persistent
// over the list).  System = one side block (CPL = false, NP = NPs) or a full coupled
// query (CPL = true, NP = 2 NPs).  Augmented matrix rows: [0, NP) the Hessian, NP the
// right-hand side v^T, NP+1..NP+15 zero, so row NP of L is y = D^-1 L^-1 v.
// L (column-major, LDR = NP + 16 rows) lives in this workgroup's scratch slab.  Per
// panel of NB columns:
//   (a) MFMA update of the panel rows from the factored columns (L streamed, D L^T of
//       the panel rows on the fly), result in LDS;
//   (b) one wave factors the NB x NB diagonal block in registers (readlane broadcasts);
//   (c) every row below solves against it in registers (barrier-free TRSM) and writes
//       its L row segment.
// Then L^T x = y in 32-column blocks from the end: a one-wave triangle per block and a
// GEMV update of the earlier entries, whose L operands are loaded behind the triangle.
// ------------------------------------------------------------------------------------
constexpr int kSolveMG = 2;     // row tiles per wave per MFMA pass
constexpr int PD = 8;           // k-steps in flight in the panel update
// solve workgroup (8 waves: 2 per SIMD, 256 VGPRs each -- the 32-wide register rows of
// the diagonal block / TRSM and the prefetch ring fit without spills)
template <int NP>
constexpr int solve_threads() { return 512; }

template <int NP>
constexpr int solve_nb() {   // 32-column panels when NP allows and LDS fits, else 16
  return NP % 32 == 0 && ((NP + 16) * 33 + NP + 32 * 32 + 64) * 8 <= 160 * 1024 ? 32 : 16;
}
template <int NP>
constexpr size_t solve_lds() {
  return (size_t)((NP + 16) * (solve_nb<NP>() + 1) + NP + solve_nb<NP>() * solve_nb<NP>() + 64) * 8;
}

__device__ __forceinline__ double readlane_dbl(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int NW>
__device__ __forceinline__ double bsum(double x, double* red) {
  x = wsum(x);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < NW; ++w) t += red[w];
  return t;
}

template <class M, int NP, bool CPL>
__global__ __launch_bounds__(solve_threads<NP>()) void k_big_solve(BigArgs A, const int32_t* __restrict__ list,
                                                   const double* __restrict__ qwork, double* __restrict__ lscr,
                                                   double* __restrict__ xb, double* __restrict__ rec) {
  constexpr int K = M::K, NPs = M::NPs, Ds = M::Ds, NB = solve_nb<NP>(), LDR = NP + 16, LDP = NB + 1;
  constexpr int NRT = LDR / 16, NCT = NB / 16, MG = kSolveMG;
  constexpr int64_t GW = gram_words<M>();
  constexpr int kST = solve_threads<NP>(), kSW = kST / 64;
  constexpr int CPT = (NP + kST - 1) / kST;    // backward-solve columns per thread
  constexpr int BW = CPT == 1 && NB == 32 ? 32 : 16;   // backward-solve block (<= NB: staged in W11)
  static_assert(BW <= NB, "backward blocks are staged in W11");
  __shared__ double P[LDR * LDP];
  __shared__ double dd[NP];
  __shared__ double W11[NB * NB];              // W11[j][jj] = L[c0+j][c0+jj] d[c0+jj], jj < j
  __shared__ double red[64];
  double* __restrict__ Ls = lscr + (int64_t)blockIdx.x * LDR * NP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ml = lane & 15, kl = lane >> 4;
  const int nsys = list[0];
  for (int w = blockIdx.x; w < nsys; w += gridDim.x) {
    const int code = list[1 + w];
    const int64_t q = CPL ? code : (code >> 1);
    const int sd = CPL ? 0 : (code & 1);
    const double* __restrict__ qw = qwork + q * M::QW;
    const double s2n = 2.0 / qw[0], cdup = qw[1], esum = qw[2];
    const double* __restrict__ vv = qw + 8 + (CPL ? 0 : sd * NPs);   // v of this system
    const int32_t u = A.qu[q], i = A.qi[q];
    const double* __restrict__ G0 = A.gram[0] + (int64_t)(A.slot[0] ? A.slot[0][u] : u) * GW;
    const double* __restrict__ G1 = A.gram[1] + (int64_t)(A.slot[1] ? A.slot[1][i] : i) * GW;
    auto aorig = [&](int r, int c) -> double {
      if (r >= NP) return (r == NP && c < NP) ? vv[c] : 0.0;
      if constexpr (!CPL) {
        if (r >= Ds || c >= Ds) return r == c ? 1.0 : 0.0;
        double h = s2n * gram_at<M>(sd ? G1 : G0, r, c);
        if (r == c) h += (M::decayed(r) ? A.wd : 0.0) + A.damping;
        return h;
      } else {
        const int sr = r >= NPs, sc = c >= NPs, rr = r - sr * NPs, cc = c - sc * NPs;
        if (rr >= Ds || cc >= Ds) return r == c ? 1.0 : 0.0;
        double h;
        if (sr == sc) {
          h = s2n * (gram_at<M>(sr ? G1 : G0, rr, cc) + cdup * vv[r] * vv[c]);
          if (r == c) h += (M::decayed(rr) ? A.wd : 0.0) + A.damping;
        } else {
          // item row / user column: 2 (cdup g_i g_u^T + esum d2r / dtheta_i dtheta_u)
          const int iu = sr ? cc : rr, ii = sr ? rr : cc;
          h = s2n * 2.0 * cdup * vv[NPs + ii] * vv[iu];
          if (ii == iu) {
            if constexpr (!M::ncf) {
              if (iu < K) h += s2n * 2.0 * esum;                                     // d2 r / dp_u dq_i = I
            } else {
              if (iu >= K) h += s2n * 2.0 * esum * (double)A.t[8][M::H + (iu - K)];    // diag(W3g)
            }
          }
        }
        return h;
      }
    };
    for (int c0 = 0; c0 < NP; c0 += NB) {
      const int rt0 = c0 >> 4, nrt = NRT - rt0;
      const int nbe = NP - c0 < NB ? NP - c0 : NB;   // last panel of NP = 16 (2m+1): one tile column
      // (a) panel rows [c0, LDR) x cols [c0, c0 + NB): A - L[:, :c0] D L[c0:c0+NB, :c0]^T
      for (int gb = wave * MG; gb < nrt; gb += kSW * MG) {
        d4_t acc[MG][NCT];
#pragma unroll
        for (int m = 0; m < MG; ++m)
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              acc[m][ct][r] = gb + m < nrt ? aorig(16 * (rt0 + gb + m) + kl + 4 * r, c0 + 16 * ct + ml) : 0.0;
        // k-steps (4 factored columns each) stream through a ring of PD register slots:
        // step s + PD is loaded while step s is multiplied (L comes from MALL/HBM)
        const int nst = c0 >> 2;
        double ra[PD][MG], rb[PD][NCT];
        auto ld = [&](int st, double (&a)[MG], double (&b)[NCT]) {
          const int kc = 4 * st + kl;
          const double* __restrict__ Lc = Ls + (int64_t)kc * LDR;
          const double dk = dd[kc];
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct) b[ct] = Lc[c0 + 16 * ct + ml] * dk;
#pragma unroll
          for (int m = 0; m < MG; ++m) a[m] = gb + m < nrt ? -Lc[16 * (rt0 + gb + m) + ml] : 0.0;
        };
#pragma unroll
        for (int d = 0; d < PD; ++d)
          if (d < nst) ld(d, ra[d], rb[d]);
        for (int s0 = 0; s0 < nst; s0 += PD) {
#pragma unroll
          for (int d = 0; d < PD; ++d) {
            if (s0 + d < nst) {
#pragma unroll
              for (int m = 0; m < MG; ++m)
                if (gb + m < nrt)
#pragma unroll
                  for (int ct = 0; ct < NCT; ++ct) acc[m][ct] = mfma4(ra[d][m], rb[d][ct], acc[m][ct]);
              if (s0 + d + PD < nst) ld(s0 + d + PD, ra[d], rb[d]);
            }
          }
        }
#pragma unroll
        for (int m = 0; m < MG; ++m)
          if (gb + m < nrt)
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
              for (int r = 0; r < 4; ++r) P[(16 * (gb + m) + kl + 4 * r) * LDP + 16 * ct + ml] = acc[m][ct][r];
      }
      __syncthreads();
      // (b) diagonal block: lane r owns row r; right-looking LDL^T with readlane broadcasts
      if (wave == 0) {
        double a[NB];
#pragma unroll
        for (int t = 0; t < NB; ++t) a[t] = lane < nbe ? P[lane * LDP + t] : (lane == t ? 1.0 : 0.0);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          // entries right of a lane's diagonal become garbage and are never read
          const double dj = readlane_dbl(a[j], j);
          const double f = lane > j ? a[j] / dj : 0.0;   // lane r > j: L[r][j]
#pragma unroll
          for (int t = j + 1; t < NB; ++t) a[t] = fma(-f, readlane_dbl(a[j], t), a[t]);
        }
        double dl = a[0];
#pragma unroll
        for (int t = 1; t < NB; ++t) dl = t == lane ? a[t] : dl;   // static indices only (no scratch)
        if (lane < nbe) {
          double* __restrict__ Wr = W11 + lane * NB;
#pragma unroll
          for (int t = 0; t < NB; ++t)
            if (t < lane) Wr[t] = a[t];
          dd[c0 + lane] = dl;
        }
        // L of the block (rows c0 + r > c0 + t): a[t] / d_t
#pragma unroll
        for (int t = 0; t < NB; ++t) {
          const double dt = readlane_dbl(dl, t);
          if (lane < nbe && t < lane) Ls[(int64_t)(c0 + t) * LDR + c0 + lane] = a[t] / dt;
        }
      }
      __syncthreads();
      // (c) rows below the block: u_j = A[r][j] - sum_{jj<j} L[r][jj] W11[j][jj],  L[r][j] = u_j / d_j
      for (int r = c0 + nbe + tid; r < LDR; r += kST) {
        double p[NB];
        const double* __restrict__ Pr = P + (r - c0) * LDP;
#pragma unroll
        for (int t = 0; t < NB; ++t) p[t] = Pr[t];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          double s = p[j];
          const double* __restrict__ Wj = W11 + j * NB;
#pragma unroll
          for (int jj = 0; jj < j; ++jj) s = fma(-p[jj], Wj[jj], s);
          p[j] = j < nbe ? s / dd[c0 + (j < nbe ? j : 0)] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < NB; ++j)
          if (j < nbe) Ls[(int64_t)(c0 + j) * LDR + r] = p[j];
      }
      __syncthreads();
    }
    // backward solve L^T x = y, y_c = L[NP][c]; BW-column blocks from the end.  Per block
    // one global round trip: the GEMV operands of the earlier columns and the block's
    // triangle (staged into W11) are loaded together, then the triangle (one wave, LDS)
    // and the GEMV update.
    double* __restrict__ xs = P;
    for (int c = tid; c < NP; c += kST) xs[c] = Ls[(int64_t)c * LDR + NP];
    for (int b0 = ((NP - 1) / BW) * BW; b0 >= 0; b0 -= BW) {
      const int bw = NP - b0 < BW ? NP - b0 : BW;
      double lv[CPT][BW];
#pragma unroll
      for (int cc = 0; cc < CPT; ++cc) {
        const int c = tid + cc * kST;
#pragma unroll
        for (int t = 0; t < BW; ++t) lv[cc][t] = (c < b0 && t < bw) ? Ls[(int64_t)c * LDR + b0 + t] : 0.0;
      }
      for (int e = tid; e < BW * BW; e += kST) {     // W11[c][t] = L[b0 + t][b0 + c], t > c
        const int cc = e / BW, t = e - cc * BW;
        W11[e] = (cc < bw && t < bw && t > cc) ? Ls[(int64_t)(b0 + cc) * LDR + b0 + t] : 0.0;
      }
      __syncthreads();
      if (wave == 0) {
        double val = lane < bw ? xs[b0 + lane] : 0.0;
        const double* __restrict__ Wc = W11 + (lane < BW ? lane : 0) * BW;
        for (int t = bw - 1; t >= 0; --t) {
          const double xt = readlane_dbl(val, t);
          if (lane < t) val = fma(-Wc[t], xt, val);
        }
        if (lane < bw) xs[b0 + lane] = val;
      }
      __syncthreads();
#pragma unroll
      for (int cc = 0; cc < CPT; ++cc) {
        const int c = tid + cc * kST;
        if (c < b0) {
          double s = xs[c];
#pragma unroll
          for (int t = 0; t < BW; ++t) s = fma(-lv[cc][t], xs[b0 + t], s);
          xs[c] = s;
        }
      }
      __syncthreads();
    }
    // epilogue: padded solution, per-side partial sums and the scoring record
    double* __restrict__ R = rec + q * M::R;
    for (int s = 0; s < (CPL ? 2 : 1); ++s) {
      const int side = CPL ? s : sd;
      const double* __restrict__ xsd = xs + (CPL ? s * NPs : 0);
      const double* __restrict__ vsd = qw + 8 + side * NPs;
      const double* __restrict__ th = qw + 8 + 2 * NPs + side * NPs;
      double* __restrict__ xo = xb + q * 2 * NPs + side * NPs;
      double cq = 0.0, xv = 0.0;
      for (int a = tid; a < NPs; a += kST) {
        const double xa = xsd[a];
        xo[a] = xa;
        if (a < Ds) {
          if (M::decayed(a)) cq = fma(xa, th[a], cq);
          xv = fma(xa, vsd[a], xv);
        }
      }
      cq = bsum<kSW>(cq, red);
      xv = bsum<kSW>(xv, red);
      double* __restrict__ S = R + 8 + side * M::SB;
      if (tid == 0) {
        R[4 + 2 * side] = A.wd * cq;
        R[5 + 2 * side] = xv;
      }
      if constexpr (!M::ncf) {
        for (int a = tid; a <= K; a += kST) S[a] = xsd[a];
        if (tid == 0) S[K + 1] = (double)(side ? u : i);
      } else {
        for (int c = tid; c < K; c += kST) {
          S[c] = xsd[c];
          S[K + c] = (double)A.t[8][M::H + c] * xsd[K + c];
        }
        if (tid == 0) S[2 * K] = (double)(side ? u : i);
      }
    }
    __syncthreads();   // xs / dd / P are rewritten by the next system
  }
}

// ------------------------------------------------------------------------------------
// Batched blocked LDL^T of the side systems (CPL = false).  The systems of a chunk are
// factored together, three launches per 64-column panel (NP % 64 != 0 ends in a
// narrower one), so thousands of independent workgroups keep every CU's memory
// pipeline busy -- the persistent one-workgroup-per-system kernel above spends most of
// its time waiting on its own panel chain.  Per system slab: L (column-major,
// LDR = NP + 16 rows, row NP the right-hand side v^T), d (NP), the current panel's
// diagonal block (64 x 64) and L11^-1 of every panel (64 x 64 each).
//   k_bs_dupd : the panel's diagonal block A - L D L^T (MFMA, k-steps split over four
//               waves);
//   k_bs_dfac : its LDL^T in one wave (readlane broadcasts), L11^-1 by forward
//               substitution (lane j: column j);
//   k_bs_trail: per 16-row tile below the block, the panel update (MFMA, L streamed)
//               and the triangular solve as one more MFMA product, P L11^-T D^-1;
//   k_bs_back : L^T x = y (y = row NP of L) by 64-column blocks from the end, each block's
//               triangle as a product with its stored L11^-1, and the scoring record.
// ------------------------------------------------------------------------------------
constexpr int kBsNB = 64;                          // panel width
constexpr int kBsMG = 2;                           // row tiles per k_bs_trail wave
constexpr int64_t kBsScratch = (int64_t)8 << 30;   // bytes of factor slabs per chunk

template <int NP>
__host__ __device__ constexpr int64_t bs_slab() {   // L, d, W, then L11^-1 of every panel
  return (int64_t)(NP + 16) * NP + NP + kBsNB * kBsNB + (int64_t)((NP + kBsNB - 1) / kBsNB) * kBsNB * kBsNB;
}

// Panel layout: when NP is not a multiple of 64 the NARROW panel comes first (columns
// [0, NP % 64)), then 64-column panels -- the narrow panel then has no update k-steps (no
// factored columns left of it), where as the last panel its k_bs_dupd / k_bs_trail were
// long single-wave chains over every earlier column for 16 columns of work (MF k = 256:
// 1.7 of 14 ms per batch).  Panel starting at column c0 keeps its L11^-1 in slot
// ceil(c0 / 64), so the first panel is slot 0 in both layouts.
__host__ __device__ constexpr int bs_first_panel(int NP) { return NP % kBsNB == 0 ? kBsNB : NP % kBsNB; }
__host__ __device__ constexpr int bs_panel_slot(int c0) { return (c0 + kBsNB - 1) / kBsNB; }

// wave-local LDS hand-off: a wave's LDS operations complete in order; this only keeps
// the compiler from moving them across the exchange
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// one side system (mf:164-251 / ncf:193-280 restricted to one side): rows/cols [0, Ds)
// (2/n) A_e + wd M + damping I, identity padding to NP, row NP the right-hand side v
template <class M, int NP>
struct SideSys {
  const double* G;
  const double* vv;
  double s2n, wd, damping;
  // branch-free (every lane loads from a valid address, then selects), so the loads of
  // a tile's elements issue back to back instead of one exec-masked round trip each
  __device__ double at(int r, int c) const {
    const bool in = r < M::Ds && c < M::Ds;
    const int rr = in ? r : 0, cc = in ? c : 0;
    const int hi = rr > cc ? rr : cc, lo = rr > cc ? cc : rr;
    const double g = G[tile_off(M::T, hi >> 4, lo >> 4) * 256 + (hi & 15) + 16 * (lo & 15)];
    const double v = vv[c < NP ? c : NP - 1];
    const double h = s2n * g + (r == c ? (M::decayed(r) ? wd : 0.0) + damping : 0.0);
    // 0/1 weights rather than selects of the loaded values (a select lets the compiler
    // sink each load into its own exec-masked branch and wait on it there)
    const double fv = (r == NP && c < NP) ? 1.0 : 0.0, fh = (r < NP && in) ? 1.0 : 0.0;
    const double fp = (r < NP && !in && r == c) ? 1.0 : 0.0;
    return fma(fv, v, fma(fh, h, fp));
  }
};

template <class M, int NP>
__device__ __forceinline__ SideSys<M, NP> side_sys(const BigArgs& A, int code, const double* __restrict__ qwork) {
  constexpr int64_t GW = gram_words<M>();
  const int64_t q = code >> 1;
  const int sd = code & 1;
  const double* __restrict__ qw = qwork + q * M::QW;
  SideSys<M, NP> S;
  S.s2n = 2.0 / qw[0];
  S.vv = qw + 8 + sd * M::NPs;
  if (sd == 0) {
    const int32_t u = A.qu[q];
    S.G = A.gram[0] + (int64_t)(A.slot[0] ? A.slot[0][u] : u) * GW;
  } else {
    const int32_t i = A.qi[q];
    S.G = A.gram[1] + (int64_t)(A.slot[1] ? A.slot[1][i] : i) * GW;
  }
  S.wd = A.wd;
  S.damping = A.damping;
  return S;
}

// diagonal block of panel c0 (NBE = 64 columns, or NP's remainder for the last panel,
// identity-padded to 64): A - L[c0:c0+NBE, :c0] D L[c0:c0+NBE, :c0]^T (lower tiles
// (rt, ct <= rt); wave w takes k-steps w, w + 4, ... through a register ring), stored
// into the slab's W area for k_bs_dfac
template <class M, int NP, int NBE>
__global__ __launch_bounds__(256) void k_bs_dupd(BigArgs A, const int32_t* __restrict__ list, int w0, int c0,
                                                 const double* __restrict__ qwork, double* __restrict__ lscr) {
  constexpr int LDR = NP + 16, NB = kBsNB, LT = NB + 1, PD = 4, NT = NBE / 16;
  __shared__ double T[NB * LT];
  const int w = w0 + (int)blockIdx.x;
  if (w >= list[0]) return;
  const SideSys<M, NP> H = side_sys<M, NP>(A, list[1 + w], qwork);
  double* __restrict__ Ls = lscr + (int64_t)blockIdx.x * bs_slab<NP>();
  const double* __restrict__ dd = Ls + (int64_t)LDR * NP;
  double* __restrict__ Dg = Ls + (int64_t)LDR * NP + NP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, ml = lane & 15, kl = lane >> 4;
#pragma unroll
  for (int i = 0; i < NB * NB / 256; ++i) {
    const int e = tid + 256 * i, r = e >> 6, cc = e & 63;
    T[r * LT + cc] = (r < NBE && cc < NBE) ? (cc <= r ? H.at(c0 + r, c0 + cc) : 0.0) : (r == cc ? 1.0 : 0.0);
  }
  d4_t acc[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) acc[t] = d4_t{0.0, 0.0, 0.0, 0.0};
  const int nst = c0 >> 2;
  const int nmy = nst > wave ? (nst - wave + 3) >> 2 : 0;
  double ra[PD][NT], rd[PD];
  auto ld = [&](int m, double (&a)[NT], double& d) {
    const int k = 4 * (wave + 4 * m) + kl;
    const double* __restrict__ Lc = Ls + (int64_t)k * LDR + c0;
    d = dd[k];
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) a[rt] = Lc[16 * rt + ml];
  };
#pragma unroll
  for (int d = 0; d < PD; ++d)
    if (d < nmy) ld(d, ra[d], rd[d]);
  for (int m0 = 0; m0 < nmy; m0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      if (m0 + d < nmy) {
        int t = 0;
#pragma unroll
        for (int rt = 0; rt < NT; ++rt) {
          const double a = -ra[d][rt] * rd[d];
#pragma unroll
          for (int ct = 0; ct <= rt; ++ct, ++t) acc[t] = mfma4(a, ra[d][ct], acc[t]);
        }
        if (m0 + d + PD < nmy) ld(m0 + d + PD, ra[d], rd[d]);
      }
    }
  }
  __syncthreads();
#pragma unroll 1
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
      int t = 0;
#pragma unroll
      for (int rt = 0; rt < NT; ++rt)
#pragma unroll
        for (int ct = 0; ct <= rt; ++ct, ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) T[(16 * rt + kl + 4 * r) * LT + 16 * ct + ml] += acc[t][r];
    }
    __syncthreads();
  }
  for (int e = tid; e < NB * NB; e += 256) Dg[e] = T[(e & 63) * LT + (e >> 6)];   // column-major
}

// LDL^T of the updated diagonal block (one wave per system; lane r owns row r, readlane
// broadcasts, no LDS), L11 and d into the slab, then L11^-1 (lane j: column j by forward
// substitution) into the panel's X slot, XOR-swizzled: Xp[n][j ^ 4 (n & 7)] = (L11^-1)[n][j],
// so k_bs_trail's B-operand reads from its linear LDS copy are two-way at most.  The
// triangular solve needs W = L11^-T D^-1, i.e. W[j][n] = Xp[n][j] / d_n: k_bs_trail scales
// its product's columns; k_bs_back uses L11^-T itself.
template <class M, int NP, int NBE>
__global__ __launch_bounds__(64) void k_bs_dfac(const int32_t* __restrict__ list, int w0, int c0,
                                                double* __restrict__ lscr) {
  constexpr int LDR = NP + 16, NB = kBsNB;
  const int w = w0 + (int)blockIdx.x;
  if (w >= list[0]) return;
  double* __restrict__ Ls = lscr + (int64_t)blockIdx.x * bs_slab<NP>();
  double* __restrict__ dd = Ls + (int64_t)LDR * NP;
  double* __restrict__ W = dd + NP;
  const int lane = threadIdx.x;
  // only the NBE x NBE block is factored (a narrow panel: the chains are NBE long); the
  // inverse is identity-padded to 64 x 64 below.  Entries right of a lane's diagonal
  // become garbage and are never read
  double a[NBE];
#pragma unroll
  for (int t = 0; t < NBE; ++t) a[t] = W[t * NB + lane];     // block stored column-major
#pragma unroll
  for (int j = 0; j < NBE; ++j) {
    const double dj = readlane_dbl(a[j], j);
    const double f = lane > j ? a[j] / dj : 0.0;
#pragma unroll
    for (int t = j + 1; t < NBE; ++t) a[t] = fma(-f, readlane_dbl(a[j], t), a[t]);
  }
  double dl = a[0];
#pragma unroll
  for (int t = 1; t < NBE; ++t) dl = t == lane ? a[t] : dl;
  if (lane < NBE) dd[c0 + lane] = dl;
  const double rdl = 1.0 / dl;
#pragma unroll
  for (int t = 0; t < NBE; ++t) {                           // a[t] becomes L11[lane][t], t < lane
    a[t] = t < lane ? a[t] * readlane_dbl(rdl, t) : 0.0;
    if (t < lane && lane < NBE) Ls[(int64_t)(c0 + t) * LDR + c0 + lane] = a[t];
  }
  // lane j: column j of L11^-1 (x_m = 0 for m < j); lanes j >= NBE: identity columns
  double x[NBE];
#pragma unroll
  for (int i = 0; i < NBE; ++i) {
    double s = i == lane ? 1.0 : 0.0;
#pragma unroll
    for (int m = 0; m < i; ++m) s = fma(-readlane_dbl(a[m], i), x[m], s);
    x[i] = s;
  }
  double* __restrict__ Xp = W + NB * NB + (int64_t)bs_panel_slot(c0) * NB * NB;
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    double xn = n == lane ? 1.0 : 0.0;
    if constexpr (NBE < NB) {
#pragma unroll
      for (int i = 0; i < NBE; ++i) xn = n == i ? x[i] : xn;
    } else {
      xn = x[n < NBE ? n : 0];
    }
    Xp[n * NB + (lane ^ (4 * (n & 7)))] = xn;
  }
}

template <class M, int NP, int NBE>
__global__ __launch_bounds__(256) void k_bs_trail(BigArgs A, const int32_t* __restrict__ list, int w0, int c0,
                                                  int tpb, int nsys, const double* __restrict__ qwork,
                                                  double* __restrict__ lscr) {
  constexpr int LDR = NP + 16, NB = kBsNB, LT = NB + 1, MG = kBsMG, PDT = 5, NT = NBE / 16;
  __shared__ double Pw[4][16 * LT];
  __shared__ double Ws[NB * NB];
  // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs, so physical block b
  // runs on XCD b % 8 (up to which XCD block 0 gets); all groups of system sys share the
  // XCD of block sys % 8, so the panel rows every group of a system reads (the B operand)
  // are one XCD's L2 lines instead of up to eight copies fetched by eight L2s
  const int xcd = (int)blockIdx.x & 7, jx = (int)blockIdx.x >> 3;
  const int sys = xcd + 8 * (jx / tpb), grp = jx % tpb;
  if (sys >= nsys) return;
  const int w = w0 + sys;
  if (w >= list[0]) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, ml = lane & 15, kl = lane >> 4;
  double* __restrict__ Ls = lscr + (int64_t)sys * bs_slab<NP>();
  const double* __restrict__ dd = Ls + (int64_t)LDR * NP;
  const double* __restrict__ W = dd + NP + NB * NB + (int64_t)bs_panel_slot(c0) * NB * NB;   // this panel's L11^-1
  // L11^-1 of this panel (k_bs_dfac) into LDS by DMA, landing while the panel update runs
#pragma unroll
  for (int i = 0; i < NB * NB / 512; ++i)
    __builtin_amdgcn_global_load_lds((glb_vp)(W + 2 * (i * 256 + tid)), (lds_vp)(Ws + 2 * (i * 256 + wave * 64)), 16,
                                     0, 0);
  const int R0 = c0 + NBE + 16 * MG * (4 * grp + wave);    // first row of this wave's tiles
  const bool active = R0 < LDR;
  const int ng = (LDR - R0) / 16 < MG ? (LDR - R0) / 16 : MG;
  const SideSys<M, NP> H = side_sys<M, NP>(A, list[1 + w], qwork);
  d4_t acc[MG][NT];
#pragma unroll
  for (int m = 0; m < MG; ++m)
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[m][ct][r] = H.at(R0 + 16 * m + kl + 4 * r, c0 + NT * ml + ct);
  // panel update: k-steps (4 factored columns each) through a ring of PDT register slots.
  // Column j of product tile ct is panel column NT j + ct, so a lane's NT B values of a
  // k-step are consecutive doubles (two 16-B loads instead of four 8-B ones)
  const int nst = active ? c0 >> 2 : 0;
  double ra[PDT][MG], rb[PDT][NT], rd[PDT];
  auto ld = [&](int st, double (&a)[MG], double (&b)[NT], double& d) {
    const int k = 4 * st + kl;
    const double* __restrict__ Lc = Ls + (int64_t)k * LDR;
    d = dd[k];
#pragma unroll
    for (int m = 0; m < MG; ++m) a[m] = Lc[R0 + 16 * m + ml];     // rows past LDR: never used (m >= ng)
    if constexpr (NT % 2 == 0) {
#pragma unroll
      for (int ct = 0; ct < NT; ct += 2) {
        const double2 v = *reinterpret_cast<const double2*>(Lc + c0 + NT * ml + ct);
        b[ct] = v.x;
        b[ct + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) b[ct] = Lc[c0 + NT * ml + ct];
    }
  };
#pragma unroll
  for (int d = 0; d < PDT; ++d)
    if (d < nst) ld(d, ra[d], rb[d], rd[d]);
  for (int s0 = 0; s0 < nst; s0 += PDT) {
#pragma unroll
    for (int d = 0; d < PDT; ++d) {
      if (s0 + d < nst) {
#pragma unroll
        for (int m = 0; m < MG; ++m) {
          const double a = -ra[d][m] * rd[d];
#pragma unroll
          for (int ct = 0; ct < NT; ++ct) acc[m][ct] = mfma4(a, rb[d][ct], acc[m][ct]);
        }
        if (s0 + d + PDT < nst) ld(s0 + d + PDT, ra[d], rb[d], rd[d]);
      }
    }
  }
  __syncthreads();   // W landed
  if (!active) return;
  // triangular solve: L[rows][panel] = P L11^-T D^-1 (upper triangular), through this
  // wave's LDS tile; column n of the product scaled by 1 / d_n
  double rdn[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) rdn[ct] = 1.0 / dd[c0 + 16 * ct + ml];
  double* __restrict__ P = Pw[wave];
#pragma unroll
  for (int m = 0; m < MG; ++m) {
    if (m >= ng) continue;
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) P[(kl + 4 * r) * LT + NT * ml + ct] = acc[m][ct][r];
    wave_lds_sync();
    double pa[4 * NT];
#pragma unroll
    for (int s = 0; s < 4 * NT; ++s) pa[s] = P[ml * LT + 4 * s + kl];
    d4_t o[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) {
      o[ct] = d4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4 * ct + 4; ++s) o[ct] = mfma4(pa[s], Ws[(16 * ct + ml) * NB + ((4 * s + kl) ^ (4 * (ml & 7)))], o[ct]);
    }
    wave_lds_sync();
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) P[(kl + 4 * r) * LT + 16 * ct + ml] = o[ct][r] * rdn[ct];
    wave_lds_sync();
    const int Rm = R0 + 16 * m;
#pragma unroll
    for (int i = 0; i < NBE / 4; ++i) Ls[(int64_t)(c0 + kl + 4 * i) * LDR + Rm + ml] = P[ml * LT + kl + 4 * i];
    wave_lds_sync();
  }
}

template <class M, int NP>
__global__ __launch_bounds__(512) void k_bs_back(BigArgs A, const int32_t* __restrict__ list, int w0,
                                                 const double* __restrict__ qwork, double* __restrict__ lscr,
                                                 double* __restrict__ xb, double* __restrict__ rec) {
  constexpr int K = M::K, NPs = M::NPs, Ds = M::Ds, LDR = NP + 16, kST = 512, kSW = kST / 64, NB = kBsNB;
  __shared__ double xs[NP + NB];       // zero past NP: a partial last block reads it unguarded
  __shared__ double red[64];
  const int w = w0 + (int)blockIdx.x;
  if (w >= list[0]) return;
  const int code = list[1 + w];
  const int64_t q = code >> 1;
  const int sd = code & 1;
  const double* __restrict__ qw = qwork + q * M::QW;
  const double* __restrict__ Ls = lscr + (int64_t)blockIdx.x * bs_slab<NP>();
  const double* __restrict__ X = Ls + (int64_t)LDR * NP + NP + NB * NB;
  const int tid = threadIdx.x;
  // L^T x = y, y_c = L[NP][c].  Per panel b from the end (64 columns; a narrow first
  // panel, bs_first_panel): x_b = L_bb^-T z_b with the panel's stored inverse (z_b: y_b after
  // the later blocks' updates), then z_c -= sum_t L[b0 + t][c] x_b[t] for every earlier c.
  // One global round trip per block.
  for (int c = tid; c < NP + NB; c += kST) xs[c] = c < NP ? Ls[(int64_t)c * LDR + NP] : 0.0;
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6;
  for (int b0 = NP - NB, bend = NP; bend > 0; bend = b0, b0 -= NB) {
    const int bw = b0 < 0 ? bend : NB;
    b0 = b0 < 0 ? 0 : b0;
    if (tid < bw) {
      // (L^-T)[c][n] = (L^-1)[n][c], zero for n < c and (identity padding) for n >= bw
      // (the padding's off-diagonal blocks are zero, so z entries past the block drop out)
      const double* __restrict__ Xb = X + (int64_t)bs_panel_slot(b0) * NB * NB;
      double xc = 0.0;
#pragma unroll 8
      for (int n = 0; n < NB; ++n) xc = fma(Xb[n * NB + (tid ^ (4 * (n & 7)))], xs[b0 + n], xc);
      __builtin_amdgcn_wave_barrier();   // (wave 0 only) every lane has read the block's z
      xs[b0 + tid] = xc;
    }
    __syncthreads();
    // z_c -= L[b0:b0+bw][c] . x_b: a column per wave step, lane t on row b0 + t (one
    // coalesced 512-B read per column), eight columns in flight
    const double xt = lane < bw ? xs[b0 + lane] : 0.0;
    for (int c0 = 8 * wave; c0 < b0; c0 += 8 * kSW) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + u;
        v[u] = (c < b0 && lane < bw) ? Ls[(int64_t)c * LDR + b0 + lane] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const double sum = wsum(v[u] * xt);
        if (lane == 0 && c0 + u < b0) xs[c0 + u] -= sum;
      }
    }
    __syncthreads();
  }
  // padded solution, this side's partial sums and scoring record (as k_big_solve)
  const int32_t u = A.qu[q], i = A.qi[q];
  const double* __restrict__ vsd = qw + 8 + sd * NPs;
  const double* __restrict__ th = qw + 8 + 2 * NPs + sd * NPs;
  double* __restrict__ xo = xb + q * 2 * NPs + sd * NPs;
  double cq = 0.0, xv = 0.0;
  for (int a = tid; a < NPs; a += kST) {
    const double xa = xs[a];
    xo[a] = xa;
    if (a < Ds) {
      if (M::decayed(a)) cq = fma(xa, th[a], cq);
      xv = fma(xa, vsd[a], xv);
    }
  }
  cq = bsum<kSW>(cq, red);
  xv = bsum<kSW>(xv, red);
  double* __restrict__ R = rec + q * M::R;
  double* __restrict__ S = R + 8 + sd * M::SB;
  if (tid == 0) {
    R[4 + 2 * sd] = A.wd * cq;
    R[5 + 2 * sd] = xv;
  }
  if constexpr (!M::ncf) {
    for (int a = tid; a <= K; a += kST) S[a] = xs[a];
    if (tid == 0) S[K + 1] = (double)(sd ? u : i);
  } else {
    for (int c = tid; c < K; c += kST) {
      S[c] = xs[c];
      S[K + c] = (double)A.t[8][M::H + c] * xs[K + c];
    }
    if (tid == 0) S[2 * K] = (double)(sd ? u : i);
  }
}

// fia_query_batch_x (a given inverse HVP, mf:210-214): the padded solution and this side's
// record words from x_in (reference theta order) instead of the k_bs_* solve -- the same
// words k_bs_back / k_big_solve write, from the prologue's theta and v.  One wave per (query, side).
template <class M>
__global__ __launch_bounds__(64) void k_big_record_x(BigArgs A, int64_t Q, const double* __restrict__ x_in,
                                                     const double* __restrict__ qwork, double* __restrict__ xb,
                                                     double* __restrict__ rec) {
  constexpr int K = M::K, NPs = M::NPs, Ds = M::Ds, D = 2 * Ds;
  const int tid = threadIdx.x;
  for (int64_t w = blockIdx.x; w < 2 * Q; w += gridDim.x) {
    const int64_t q = w >> 1;
    const int sd = (int)(w & 1);
    const double* __restrict__ qw = qwork + q * M::QW;
    const double* __restrict__ vsd = qw + 8 + sd * NPs;
    const double* __restrict__ th = qw + 8 + 2 * NPs + sd * NPs;
    const double* __restrict__ xq = x_in + q * D;
    double* __restrict__ xo = xb + q * 2 * NPs + sd * NPs;
    double* __restrict__ R = rec + q * M::R;
    double* __restrict__ S = R + 8 + sd * M::SB;
    double cq = 0.0, xv = 0.0;
    for (int a = tid; a < NPs; a += 64) {
      const double xa = a < Ds ? xq[M::ref_index(sd, a)] : 0.0;
      xo[a] = xa;
      if (a < Ds) {
        if (M::decayed(a)) cq = fma(xa, th[a], cq);
        xv = fma(xa, vsd[a], xv);
      }
      if constexpr (!M::ncf) {
        if (a <= K) S[a] = xa;
      } else {
        if (a < K) S[a] = xa;
        else if (a < Ds) S[a] = (double)A.t[8][M::H + (a - K)] * xa;
      }
    }
    cq = wsum(cq);
    xv = wsum(xv);
    if (tid == 0) {
      R[4 + 2 * sd] = A.wd * cq;
      R[5 + 2 * sd] = xv;
      const int32_t u = A.qu[q], i = A.qi[q];
      S[M::ncf ? 2 * K : K + 1] = (double)(sd ? u : i);
    }
  }
}

// per-query record header and x in the reference theta order
template <class M>
__global__ __launch_bounds__(64) void k_big_finish(int64_t Q, const double* __restrict__ qwork,
                                                   const double* __restrict__ xb, double* __restrict__ rec,
                                                   double* __restrict__ x_out) {
  constexpr int Ds = M::Ds, NPs = M::NPs, D = 2 * Ds;
  for (int64_t q = blockIdx.x; q < Q; q += gridDim.x) {
    const double n = qwork[q * M::QW];
    double* R = rec + q * M::R;
    if (threadIdx.x == 0) {
      R[0] = n > 0.0 ? 1.0 / n : NAN;
      if (n > 0.0) {
        R[1] = R[4] + R[6];
        R[2] = R[5] + R[7];
        R[3] = qwork[q * M::QW + 3];
      }
    }
    if (x_out)
      for (int a = threadIdx.x; a < D; a += 64) {
        const int side = a >= Ds, aa = a - side * Ds;
        x_out[q * D + M::ref_index(side, aa)] = n > 0.0 ? xb[q * 2 * NPs + side * NPs + aa] : NAN;
      }
  }
}

// ------------------------------------------------------------------------------------
// Entity-shared scoring on the f64 matrix cores (work items from build_groups: one
// <= kChunk chunk of one entity's list x one block of <= kBigMfmaQB = 32 queries with that
// entity).  Per rating:
//   MF  s_q = x_emb,q . emb_other + x_bias,q
//   NCF s_q = x_mlp,q . g_mlp,j + (W3g * x_gmf,q) . gmf_other
//   influence = (2 e_j s_q + c_q) / n_q   (mf:240-246); the test pair's own train row
//   takes e and s = x.v from the record (bit-identical copies).  A workgroup
// takes one work item; wave h is scoring pass h (ratings [64 h, 64 h + 64) of the
// chunk, four 16-rating tiles).  Per tile the scores are 16 x 16 MFMA products over the
// dotted length KD (MF: x_emb . emb_other; NCF: x_mlp . g_mlp,j then (W3g * x_gmf) .
// gmf_other): A = a 16-query half of the block's query vectors (LDS, k-major), B = the
// tile's rating vectors streamed from HBM, four consecutive coordinates per lane (full
// 128-B lines per row).  A block of more than 16 queries runs both halves on each loaded
// B operand, so a rating row is read once per 32 queries (the k = 256 rows are 1-3 KB).
// The LDS holds one K-coordinate segment of the 32 query vectors at a time (NCF: the
// x_mlp half, then the W3g * x_gmf half): 67.6 KB at k = 256, two workgroups per CU.
// Lane (m, g) ends with the scores of rating m against queries g, g + 4, g + 8, g + 12 of
// each half, so each influence store is four 128-B segments.
// ------------------------------------------------------------------------------------
constexpr int kBigMfmaQB = 32;

template <class M>
constexpr int score_kd() { return M::ncf ? 2 * M::K : M::K; }

template <class M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_big_score_mfma(
    BigArgs A, int64_t nE, const int64_t* __restrict__ wstart, const int32_t* __restrict__ witems,
    const int64_t* __restrict__ gstart, const int32_t* __restrict__ gq, const int64_t* __restrict__ qbase,
    const double* __restrict__ rec, int32_t* __restrict__ rel_idx, double* __restrict__ influence, int K_top,
    int32_t* __restrict__ cand_pos, double* __restrict__ cand_val) {
  constexpr int K = M::K, QB = kBigMfmaQB, XS = QB + 1, NPASS = kScoreRows;
  static_assert(NPASS == 4 && QB == 32, "one wave per scoring pass, two 16-query halves");
  __shared__ double Xs[K * XS];        // Xs[k * XS + j]: coordinate seg + k of query j's vector
  __shared__ double Qs[QB][6];         // 1/n, c_q, x.v, r-hat, dup_other, x_bias (MF)
  __shared__ int64_t Bs[QB][3];        // influence offset, candidate chunk, position offset
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, ml = lane & 15, kl = lane >> 4;
  const int64_t n_items = wstart[nE];
  for (int64_t wi = blockIdx.x; wi < n_items; wi += gridDim.x) {
    const int32_t g = witems[3 * wi], cidx = witems[3 * wi + 1], qblk = witems[3 * wi + 2];
    const int sd = g >= A.U ? 1 : 0;
    const int32_t e = sd ? (int32_t)(g - A.U) : g;
    const int64_t lb = A.ptr[sd][e] + (int64_t)cidx * kChunk;
    const int64_t rem = A.ptr[sd][e + 1] - lb;
    const int len = rem < kChunk ? (int)rem : kChunk;
    const int64_t gb = gstart[g] + (int64_t)qblk * QB;
    const int64_t gn = gstart[g + 1] - gb;
    const int nq = gn < QB ? (int)gn : QB;
    // coordinates [seg, seg + K) of the block's side vectors into Xs (zero past nq)
    auto stage = [&](int seg) {
      for (int t = tid; t < K * QB; t += 256) {
        const int j = t / K, k = t - j * K;
        double v = 0.0;
        if (j < nq) v = rec[(int64_t)gq[gb + j] * M::R + 8 + sd * M::SB + seg + k];
        Xs[k * XS + j] = v;
      }
    };
    __syncthreads();                   // the previous item's LDS is consumed
    stage(0);
    if (tid < QB) {
      const int32_t q = gq[gb + (tid < nq ? tid : nq - 1)];
      const double* __restrict__ R = rec + (int64_t)q * M::R;
      const double* __restrict__ S = R + 8 + sd * M::SB;
      Qs[tid][0] = R[0];
      Qs[tid][1] = R[1];
      Qs[tid][2] = R[2];
      Qs[tid][3] = R[3];
      Qs[tid][4] = M::ncf ? S[2 * K] : S[K + 1];
      Qs[tid][5] = M::ncf ? 0.0 : S[K];
      const int64_t* qb = qbase + 4 * (int64_t)q;
      Bs[tid][0] = qb[sd] + (int64_t)cidx * kChunk;
      Bs[tid][1] = qb[2 + sd] + cidx;
      Bs[tid][2] = sd ? qb[1] - qb[0] : 0;
    }
    __syncthreads();
    // this wave's four tiles: rating idx = 64 wave + 16 t + m
    int32_t o[4], rw[4];
    float y[4];
    double ej[4];
    bool ok[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int idx = 64 * wave + 16 * t + ml;
      ok[t] = idx < len;
      const int li = ok[t] ? idx : 0;
      o[t] = A.other[sd][lb + li];
      rw[t] = A.row[sd][lb + li];
      y[t] = A.rating[sd][lb + li];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) ej[t] = A.resid[rw[t]];
    d4_t acc[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[h][t] = d4_t{0.0, 0.0, 0.0, 0.0};
    // the MFMA passes over one staged segment; TWO: both 16-query halves per B operand
    // (a uniform branch around whole passes, none inside the MFMA chains)
    auto segment = [&](auto two, auto seg) {
      constexpr bool TWO = decltype(two)::value;
      constexpr bool GM = M::ncf && decltype(seg)::value == 0;   // the g_mlp segment
      // k-groups of 16 coordinates: lane (m, g) holds coordinates 16 G + 4 g + i, i < 4,
      // of rating m; MFMA step i of the group uses coordinate 16 G + 4 g + i on both sides
      auto group = [&](int G, const double (&b)[4][4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double* __restrict__ xr = Xs + (16 * G + 4 * kl + i) * XS + ml;
          const double a0 = xr[0];
          const double a1 = TWO ? xr[16] : 0.0;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            acc[0][t] = mfma4(a0, b[t][i], acc[0][t]);
            if constexpr (TWO) acc[1][t] = mfma4(a1, b[t][i], acc[1][t]);
          }
        }
      };
      if constexpr (GM) {
        // x_mlp . g_mlp,j: g_mlp rows of this side (fp64)
        const double* __restrict__ gmr[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) gmr[t] = A.gm[sd] + (int64_t)rw[t] * K + 4 * kl;
        double bA[4][4], bB[4][4];
        auto ldg = [&](int G, double (&b)[4][4]) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const double2 u0 = *reinterpret_cast<const double2*>(gmr[t] + 16 * G);
            const double2 u1 = *reinterpret_cast<const double2*>(gmr[t] + 16 * G + 2);
            b[t][0] = u0.x; b[t][1] = u0.y; b[t][2] = u1.x; b[t][3] = u1.y;
          }
        };
        ldg(0, bA);
        for (int G = 0; G < K / 16; G += 2) {
          ldg(G + 1, bB);
          group(G, bA);
          if (G + 2 < K / 16) ldg(G + 2, bA);
          group(G + 1, bB);
        }
      } else {
        // (MF: x_emb, NCF: W3g * x_gmf) . the other side's embedding row (fp32)
        const float* __restrict__ T = M::ncf ? (sd == 0 ? A.t[3] : A.t[2]) : (sd == 0 ? A.t[1] : A.t[0]);
        const float* __restrict__ er[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) er[t] = T + (int64_t)o[t] * K + 4 * kl;
        float4 fA[4], fB[4];
        auto lde = [&](int G, float4 (&f)[4]) {
#pragma unroll
          for (int t = 0; t < 4; ++t) f[t] = *reinterpret_cast<const float4*>(er[t] + 16 * G);
        };
        auto grp = [&](int G, const float4 (&f)[4]) {
          double b[4][4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            b[t][0] = f[t].x; b[t][1] = f[t].y; b[t][2] = f[t].z; b[t][3] = f[t].w;
          }
          group(G, b);
        };
        lde(0, fA);
        for (int G = 0; G < K / 16; G += 2) {
          lde(G + 1, fB);
          grp(G, fA);
          if (G + 2 < K / 16) lde(G + 2, fA);
          grp(G + 1, fB);
        }
      }
    };
    const bool two = nq > 16;
    auto passes = [&](auto seg) {
      if (two) segment(std::integral_constant<bool, true>{}, seg);
      else segment(std::integral_constant<bool, false>{}, seg);
    };
    passes(std::integral_constant<int, 0>{});
    if constexpr (M::ncf) {
      __syncthreads();                 // every wave is done with the x_mlp segment
      stage(K);
      __syncthreads();
      passes(std::integral_constant<int, 1>{});
    }
    // influence of rating m against queries h0 + kl + 4 r of one half
    auto epilogue = [&](d4_t (&ac)[4], int h0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = h0 + kl + 4 * r;
        const double inv_n = Qs[j][0], cq = Qs[j][1], xv = Qs[j][2], rhat = Qs[j][3], dup = Qs[j][4], xb = Qs[j][5];
        const int64_t obj = Bs[j][0];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          double ss = ac[t][r] + xb, ee = ej[t];
          if ((double)o[t] == dup) { ee = rhat - (double)y[t]; ss = xv; }
          const double infl = (2.0 * ee * ss + cq) * inv_n;
          const int idx = 64 * wave + 16 * t + ml;
          if (ok[t] && j < nq) {
            if (influence) influence[obj + idx] = infl;
            if (rel_idx) rel_idx[obj + idx] = rw[t];
          }
          ac[t][r] = infl;
        }
      }
      if (K_top > 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = h0 + kl + 4 * r;
          const int64_t cbj = Bs[j][1], poj = Bs[j][2];
          double pa = INFINITY;
          int pp = -1;
          for (int tt = 0; tt < K_top; ++tt) {
            double ba = -2.0, bv = 0.0;
            int bp = 0x7fffffff;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int lp = ok[t] ? cidx * kChunk + 64 * wave + 16 * t + ml : -1;
              const double key = topk_key(ac[t][r]);     // (recomputed: no key registers)
              if (lp >= 0 && better(pa, pp, key, lp) && better(key, lp, ba, bp)) {
                ba = key;
                bp = lp;
                bv = ac[t][r];
              }
            }
#pragma unroll
            for (int off = 8; off > 0; off >>= 1) {   // within the 16 lanes of query j
              const double oa = __shfl_xor(ba, off);
              const int op = __shfl_xor(bp, off);
              const double ov = __shfl_xor(bv, off);
              if (better(oa, op, ba, bp)) { ba = oa; bp = op; bv = ov; }
            }
            if (ml == 0 && j < nq) {
              const bool okk = ba > -1.5;
              const int64_t slot = (cbj * NPASS + wave) * K_top + tt;
              cand_pos[slot] = okk ? (int32_t)(bp + poj) : -1;
              cand_val[slot] = okk ? bv : NAN;
            }
            pa = ba;
            pp = bp;
          }
        }
      }
    };
    epilogue(acc[0], 0);
    if (two) epilogue(acc[1], 16);
  }
}

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
BigArgs make_big_args(fia_ctx* c, const int32_t* qu, const int32_t* qi) {
  BigArgs A;
  A.qu = qu;
  A.qi = qi;
  A.U = c->p.U;
  A.I = c->p.I;
  for (int s = 0; s < 2; ++s) {
    A.ptr[s] = c->idx.side[s].ptr.as<int64_t>();
    A.row[s] = c->idx.side[s].row.as<int32_t>();
    A.other[s] = c->idx.side[s].other.as<int32_t>();
    A.rating[s] = c->idx.side[s].rating.as<float>();
    A.gram[s] = c->gram[s].as<double>();
    A.l1[s] = c->l1[s].as<double>();
    A.gm[s] = c->gm[s].as<double>();
    A.slot[s] = c->subset ? c->slot[s].as<int32_t>() : nullptr;
  }
  A.resid = c->resid.as<double>();
  for (int t = 0; t < 10; ++t) A.t[t] = c->p.t[t];
  A.wd = c->p.wd;
  A.damping = c->p.damping;
  A.pairs.key = c->idx.pkey.as<unsigned long long>();
  A.pairs.cnt = c->idx.pcnt.as<int32_t>();
  A.pairs.sum = c->idx.psum.as<double>();
  A.pairs.mask = (unsigned long long)(c->idx.pcap - 1);
  return A;
}

inline unsigned grid_cap(int64_t n, int64_t cap) {
  if (n < 1) n = 1;
  return (unsigned)(n < cap ? n : cap);
}

int cu_count(fia_ctx* c) {
  if (c->num_cus <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || n <= 0) n = 256;
    c->num_cus = n;
  }
  return c->num_cus;
}

// Gram work lists: slices of <= kBigSlice ratings of every cached entity, longest lists
// first; items {entity, start, len, dst} with dst >= 0 the cache slot, dst < 0 the partial
// slot -dst-1 of a split list; split lists get a combine entry {cache slot, first partial,
// n partials, 0} summed in slot order.  marks == nullptr: every entity, slot = entity id
// (lists cached per index); else only the marked entities, numbered in entity order.
hipError_t big_work_lists(fia_ctx* c, const std::vector<uint8_t>* marks, hipStream_t s) {
  Index& X = c->idx;
  if (!marks && !c->subset && c->bitems_version == X.version) return hipSuccess;
  for (int sd = 0; sd < 2; ++sd) {
    const std::vector<int64_t>& hp = X.hptr[sd];
    const int64_t ne = (int64_t)hp.size() - 1;
    std::vector<int32_t> slot((size_t)ne, -1);
    int32_t ncache = 0;
    for (int64_t e = 0; e < ne; ++e)
      if (!marks || marks[sd][(size_t)e]) slot[(size_t)e] = ncache++;
    std::vector<int32_t> items, comb;
    int32_t parts = 0;
    for (int32_t e : X.hord[sd]) {
      if (slot[(size_t)e] < 0) continue;
      const int64_t len = hp[(size_t)e + 1] - hp[(size_t)e];
      const int64_t nit = len == 0 ? 1 : (len + kBigSlice - 1) / kBigSlice;
      if (nit > 1) comb.insert(comb.end(), {slot[(size_t)e], parts, (int32_t)nit, 0});
      for (int64_t t = 0; t < nit; ++t) {
        const int64_t st = t * kBigSlice;
        const int64_t ln = std::min<int64_t>(kBigSlice, len - st);
        const int32_t dst = nit > 1 ? -(1 + parts++) : slot[(size_t)e];
        items.insert(items.end(), {e, (int32_t)st, (int32_t)(ln < 0 ? 0 : ln), dst});
      }
    }
    c->n_bitems[sd] = (int64_t)items.size() / 4;
    c->n_bcomb[sd] = (int64_t)comb.size() / 4;
    c->n_bslots[sd] = parts;
    c->n_bcache[sd] = ncache;
    if (!items.empty()) {
      FIA_HIP_TRY(c->bitems[sd].reserve(sizeof(int32_t) * items.size(), s));
      FIA_HIP_TRY(hipMemcpyAsync(c->bitems[sd].ptr, items.data(), sizeof(int32_t) * items.size(), hipMemcpyHostToDevice, s));
    }
    if (!comb.empty()) {
      FIA_HIP_TRY(c->bcomb[sd].reserve(sizeof(int32_t) * comb.size(), s));
      FIA_HIP_TRY(hipMemcpyAsync(c->bcomb[sd].ptr, comb.data(), sizeof(int32_t) * comb.size(), hipMemcpyHostToDevice, s));
    }
    if (marks) {
      FIA_HIP_TRY(c->slot[sd].reserve(sizeof(int32_t) * (size_t)(ne + 1), s));
      FIA_HIP_TRY(hipMemcpyAsync(c->slot[sd].ptr, slot.data(), sizeof(int32_t) * slot.size(), hipMemcpyHostToDevice, s));
    }
    FIA_HIP_TRY(hipStreamSynchronize(s));   // this side's host lists are freed at the end of the iteration
  }
  c->bitems_version = marks ? ~0ull : X.version;
  c->subset = marks != nullptr;
  return hipSuccess;
}

template <class M>
hipError_t prepare_big_impl(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, hipStream_t s) {
  constexpr int K = M::K;
  constexpr int64_t GW = gram_words<M>();
  Index& X = c->idx;
  const int64_t N = X.N;
  const int64_t n_ent[2] = {c->p.U, c->p.I};
  const unsigned gN = grid_cap((N + 255) / 256, 16384);
  // entity selection first (host round trip), so a too-large cache fails before any work
  std::vector<uint8_t> marks[2];
  if (qu) {
    FIA_HIP_TRY(c->mark.reserve((size_t)(n_ent[0] + n_ent[1]), s));
    FIA_HIP_TRY(hipMemsetAsync(c->mark.ptr, 0, (size_t)(n_ent[0] + n_ent[1]), s));
    if (Q > 0) {
      hipLaunchKernelGGL(k_mark, dim3(grid_cap((Q + 255) / 256, 4096)), dim3(256), 0, s, Q, qu, qi, n_ent[0],
                         n_ent[1], c->mark.as<uint8_t>());
      FIA_HIP_TRY(hipGetLastError());
    }
    marks[0].resize((size_t)n_ent[0]);
    marks[1].resize((size_t)n_ent[1]);
    FIA_HIP_TRY(hipMemcpyAsync(marks[0].data(), c->mark.ptr, (size_t)n_ent[0], hipMemcpyDeviceToHost, s));
    FIA_HIP_TRY(hipMemcpyAsync(marks[1].data(), c->mark.as<uint8_t>() + n_ent[0], (size_t)n_ent[1],
                               hipMemcpyDeviceToHost, s));
    FIA_HIP_TRY(hipStreamSynchronize(s));
  }
  FIA_HIP_TRY(big_work_lists(c, qu ? marks : nullptr, s));
  FIA_HIP_TRY(ensure_self(c, s));
  FIA_HIP_TRY(c->resid.reserve(sizeof(double) * (size_t)(N + 1), s));
  if constexpr (!M::ncf) {
    if (N > 0) {
      hipLaunchKernelGGL(k_resid_mf<K>, dim3(gN), dim3(256), 0, s, N, c->self[0].as<int32_t>(),
                         X.side[0].other.as<int32_t>(), X.side[0].row.as<int32_t>(), X.side[0].rating.as<float>(),
                         c->p.t[0], c->p.t[1], c->p.t[2], c->p.t[3], c->p.t[4], c->resid.as<double>(),
                         qu ? c->mark.as<uint8_t>() : nullptr, n_ent[0]);
      FIA_HIP_TRY(hipGetLastError());
    }
  } else {
    for (int sd = 0; sd < 2; ++sd) {
      FIA_HIP_TRY(c->l1[sd].reserve(sizeof(double) * (size_t)(n_ent[sd] * K + 1), s));
      hipLaunchKernelGGL(k_l1_big<K>, dim3(grid_cap((n_ent[sd] * K + 255) / 256, 16384)), dim3(256), 0, s,
                         c->p.t[sd], c->p.t[4], sd * K, n_ent[sd], c->l1[sd].as<double>());
      FIA_HIP_TRY(hipGetLastError());
      FIA_HIP_TRY(c->gm[sd].reserve(sizeof(double) * (size_t)(N * K + 1), s));
    }
    FIA_HIP_TRY(c->wfrag.reserve(sizeof(double) * (size_t)3 * K * K, s));
    hipLaunchKernelGGL(k_ncf_wfrag<K>, dim3(3 * K * K / 256), dim3(256), 0, s, c->p.t[4], c->p.t[6],
                       c->wfrag.as<double>());
    FIA_HIP_TRY(hipGetLastError());
    for (int pass = qu ? 0 : -1; N > 0 && pass < (qu ? 2 : 0); ++pass) {
      const int sd = pass < 0 ? 0 : pass;
      hipLaunchKernelGGL(k_ncf_rows<K>, dim3(grid_cap((N + 15) / 16, 65536)), dim3(64 * kRowWaves), 0, s, N, pass,
                         c->self[sd].as<int32_t>(), X.side[sd].other.as<int32_t>(), X.side[sd].row.as<int32_t>(),
                         X.side[sd].rating.as<float>(), c->l1[0].as<double>(), c->l1[1].as<double>(), c->p.t[5],
                         c->p.t[6], c->p.t[7], c->p.t[8], c->p.t[9], c->p.t[2], c->p.t[3],
                         c->wfrag.as<const double2>(), c->gm[0].as<double>(), c->gm[1].as<double>(), c->resid.as<double>(),
                         qu ? c->mark.as<uint8_t>() : (const uint8_t*)nullptr, n_ent[0]);
      FIA_HIP_TRY(hipGetLastError());
    }
  }
  for (int sd = 0; sd < 2; ++sd) {
    FIA_HIP_TRY(c->gram[sd].reserve(sizeof(double) * (size_t)((c->n_bcache[sd] > 0 ? c->n_bcache[sd] : 1) * GW), s));
    if (c->n_bslots[sd] > 0) FIA_HIP_TRY(c->gpart[sd].reserve(sizeof(double) * (size_t)(c->n_bslots[sd] * GW), s));
    const float* emb_other = M::ncf ? c->p.t[sd == 0 ? 3 : 2] : c->p.t[sd == 0 ? 1 : 0];
    if (c->n_bitems[sd] > 0) {
      constexpr int64_t NG = GramCfg<M>::NG, unit = 8 * NG;
      const int64_t n_vb = (c->n_bitems[sd] + 7) / 8 * unit;
      const dim3 g_gram = NG > 2 ? dim3((unsigned)(n_vb < (1 << 20) / unit * unit ? n_vb : (1 << 20) / unit * unit))
                                 : dim3(grid_cap(c->n_bitems[sd], 1 << 20), (unsigned)NG);
      hipLaunchKernelGGL(k_big_gram<M>, g_gram, dim3(64 * kGW), 0, s,
                         sd, c->n_bitems[sd], c->bitems[sd].as<int32_t>(), X.side[sd].ptr.as<int64_t>(),
                         X.side[sd].other.as<int32_t>(), X.side[sd].row.as<int32_t>(), emb_other,
                         c->gm[sd].as<double>(), c->p.t[8], c->gram[sd].as<double>(), c->gpart[sd].as<double>());
      FIA_HIP_TRY(hipGetLastError());
    }
    if (c->n_bcomb[sd] > 0) {
      hipLaunchKernelGGL(k_big_combine, dim3(grid_cap(c->n_bcomb[sd], 1024), kCombSplit), dim3(256), 0, s, c->n_bcomb[sd],
                         c->bcomb[sd].as<int32_t>(), GW, c->gpart[sd].as<double>(), c->gram[sd].as<double>());
      FIA_HIP_TRY(hipGetLastError());
    }
  }
  return hipSuccess;
}

template <class M, int NP, bool CPL>
hipError_t launch_solve(fia_ctx* c, const BigArgs& A, int64_t max_sys, const int32_t* list, hipStream_t s) {
  if (max_sys <= 0) return hipSuccess;
  constexpr size_t lds = solve_lds<NP>();
  const int per_cu = (int)((160 * 1024) / lds);
  const int64_t resident = (int64_t)cu_count(c) * (per_cu > 0 ? per_cu : 1);
  const int64_t grid = max_sys < resident ? max_sys : resident;
  constexpr int64_t slab = (int64_t)(NP + 16) * NP;
  FIA_HIP_TRY(c->lscr.reserve(sizeof(double) * (size_t)(grid * slab), s));
  hipLaunchKernelGGL((k_big_solve<M, NP, CPL>), dim3((unsigned)grid), dim3(solve_threads<NP>()), 0, s, A, list,
                     c->qwork.as<double>(), c->lscr.as<double>(), c->xb.as<double>(), c->rec.as<double>());
  return hipGetLastError();
}

// side systems through the batched panel kernels, chunks of <= kBsScratch bytes of slabs;
// list[0] (the device-side count) bounds every launch, max_sys only sizes them
template <class M, int NP, int NBE>
hipError_t launch_bs_panel(fia_ctx* c, const BigArgs& A, int64_t w0, int64_t n, int c0, const int32_t* list,
                           hipStream_t s) {
  hipLaunchKernelGGL((k_bs_dupd<M, NP, NBE>), dim3((unsigned)n), dim3(256), 0, s, A, list, (int)w0, c0,
                     c->qwork.as<double>(), c->lscr.as<double>());
  FIA_HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL((k_bs_dfac<M, NP, NBE>), dim3((unsigned)n), dim3(64), 0, s, list, (int)w0, c0,
                     c->lscr.as<double>());
  FIA_HIP_TRY(hipGetLastError());
  const int tiles = (NP + 16 - c0 - NBE) / 16;
  const int tpb = (tiles + 4 * kBsMG - 1) / (4 * kBsMG);
  hipLaunchKernelGGL((k_bs_trail<M, NP, NBE>), dim3((unsigned)(8 * ((n + 7) / 8) * tpb)), dim3(256), 0, s, A, list,
                     (int)w0, c0, tpb, (int)n, c->qwork.as<double>(), c->lscr.as<double>());
  return hipGetLastError();
}

template <class M, int NP>
hipError_t launch_solve_batched(fia_ctx* c, const BigArgs& A, int64_t max_sys, const int32_t* list, hipStream_t s) {
  static_assert(NP % 16 == 0, "side blocks are whole 16-column tiles");
  constexpr int kFirst = bs_first_panel(NP);   // first panel's width
  if (max_sys <= 0) return hipSuccess;
  constexpr int64_t slab = bs_slab<NP>();
  int64_t S = kBsScratch / (int64_t)(sizeof(double) * slab);
  S = S < 1 ? 1 : (S > max_sys ? max_sys : S);
  FIA_HIP_TRY(c->lscr.reserve(sizeof(double) * (size_t)(S * slab), s));
  for (int64_t w0 = 0; w0 < max_sys; w0 += S) {
    const int64_t n = max_sys - w0 < S ? max_sys - w0 : S;
    // the narrow panel (if any) first, then 64-column panels (bs_first_panel)
    FIA_HIP_TRY((launch_bs_panel<M, NP, kFirst>(c, A, w0, n, 0, list, s)));
    for (int c0 = kFirst; c0 < NP; c0 += kBsNB) FIA_HIP_TRY((launch_bs_panel<M, NP, kBsNB>(c, A, w0, n, c0, list, s)));
    hipLaunchKernelGGL((k_bs_back<M, NP>), dim3((unsigned)n), dim3(512), 0, s, A, list, (int)w0,
                       c->qwork.as<double>(), c->lscr.as<double>(), c->xb.as<double>(), c->rec.as<double>());
    FIA_HIP_TRY(hipGetLastError());
  }
  return hipSuccess;
}

template <class M>
hipError_t query_big_impl(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                          int64_t max_chunks, int32_t* rel_idx, double* influence, double* x_out, int K,
                          int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s,
                          const double* x_in) {
  constexpr int NPs = M::NPs, NPASS = kScoreRows;
  FIA_HIP_TRY(c->rec.reserve(sizeof(double) * (size_t)(Q * M::R + 1), s));
  FIA_HIP_TRY(c->qwork.reserve(sizeof(double) * (size_t)(Q * M::QW + 1), s));
  FIA_HIP_TRY(c->xb.reserve(sizeof(double) * (size_t)(Q * 2 * NPs + 1), s));
  FIA_HIP_TRY(c->syslist.reserve(sizeof(int32_t) * (size_t)(2 * Q + 2), s));
  FIA_HIP_TRY(c->cpllist.reserve(sizeof(int32_t) * (size_t)(Q + 2), s));
  if (K > 0) {
    FIA_HIP_TRY(c->cand_pos.reserve(sizeof(int32_t) * (size_t)((max_chunks + 1) * K * NPASS), s));
    FIA_HIP_TRY(c->cand_val.reserve(sizeof(double) * (size_t)((max_chunks + 1) * K * NPASS), s));
  }
  const BigArgs A = make_big_args(c, qu, qi);
  phase_begin(c, 4, s);
  FIA_HIP_TRY(build_chunks(c, Q, qu, qi, offsets, max_chunks, true, s));
  FIA_HIP_TRY(build_groups(c, Q, qu, qi, offsets, max_chunks, kBigMfmaQB, s));
  phase_end(c, 4, s);
  phase_begin(c, 1, s);
  FIA_HIP_TRY(hipMemsetAsync(c->syslist.ptr, 0, sizeof(int32_t), s));
  FIA_HIP_TRY(hipMemsetAsync(c->cpllist.ptr, 0, sizeof(int32_t), s));
  hipLaunchKernelGGL(k_big_prologue<M>, dim3(grid_cap(Q, 1 << 20)), dim3(256), 0, s, A, Q, c->qwork.as<double>(),
                     c->syslist.as<int32_t>(), c->cpllist.as<int32_t>());
  FIA_HIP_TRY(hipGetLastError());
  if (x_in) {
    // a given inverse HVP: the records straight from it, no solve (fia_query_batch_x)
    if (Q > 0)
      hipLaunchKernelGGL(k_big_record_x<M>, dim3(grid_cap(2 * Q, 1 << 20)), dim3(64), 0, s, A, Q, x_in,
                         (const double*)c->qwork.as<double>(), c->xb.as<double>(), c->rec.as<double>());
    FIA_HIP_TRY(hipGetLastError());
  } else {
    FIA_HIP_TRY((launch_solve_batched<M, NPs>(c, A, 2 * Q, c->syslist.as<int32_t>(), s)));
    FIA_HIP_TRY((launch_solve<M, 2 * NPs, true>(c, A, Q, c->cpllist.as<int32_t>(), s)));
  }
  hipLaunchKernelGGL(k_big_finish<M>, dim3(grid_cap(Q, 1 << 20)), dim3(64), 0, s, Q, c->qwork.as<double>(),
                     c->xb.as<double>(), c->rec.as<double>(), x_out);
  FIA_HIP_TRY(hipGetLastError());
  phase_end(c, 1, s);
  const PhaseSpan span = phase_span(c, 2);
  hipExtLaunchKernelGGL(k_big_score_mfma<M>, dim3(grid_cap(max_chunks, 8192)), dim3(256), 0, s, span.a, span.b, 0, A,
                        c->p.U + c->p.I, c->wstart.as<int64_t>(), c->witems.as<int32_t>(), c->gstart.as<int64_t>(),
                        c->gq.as<int32_t>(), c->qbase.as<int64_t>(), c->rec.as<double>(), rel_idx, influence, K,
                        c->cand_pos.as<int32_t>(), c->cand_val.as<double>());
  FIA_HIP_TRY(hipGetLastError());
  if (K > 0) {
    phase_begin(c, 3, s);
    FIA_HIP_TRY(launch_topk_merge(c, Q, qu, qi, K, NPASS, topk_pos, topk_idx, topk_val, s, max_chunks));
    phase_end(c, 3, s);
  }
  return hipSuccess;
}

}  // namespace

#define FIA_BIG_CASES(X) \
  X(FIA_MODEL_MF, 128, BMF<128>) X(FIA_MODEL_MF, 256, BMF<256>) X(FIA_MODEL_NCF, 64, BNCF<64>) \
  X(FIA_MODEL_NCF, 128, BNCF<128>) X(FIA_MODEL_NCF, 256, BNCF<256>)

// per-list-position owning entity of both sides (rebuilt when the index changes)
hipError_t ensure_self(fia_ctx* c, hipStream_t s) {
  const Index& X = c->idx;
  if (c->self_version == X.version) return hipSuccess;
  const int64_t N = X.N, n_ent[2] = {X.U, X.I};
  for (int sd = 0; sd < 2; ++sd) {
    FIA_HIP_TRY(c->self[sd].reserve(sizeof(int32_t) * (size_t)(N + 1), s));
    if (N > 0) {
      hipLaunchKernelGGL(k_self, dim3(grid_cap((N + 255) / 256, 65536)), dim3(256), 0, s, N, n_ent[sd],
                         X.side[sd].ptr.as<int64_t>(), c->self[sd].as<int32_t>());
      FIA_HIP_TRY(hipGetLastError());
    }
  }
  c->self_version = X.version;
  return hipSuccess;
}

bool big_supported(int model, int k) {
#define X(m, kk, T) if (model == m && k == kk) return true;
  FIA_BIG_CASES(X)
#undef X
  return false;
}

hipError_t prepare_big(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, hipStream_t s) {
  c->small_subset = false;
#define X(m, kk, T) if (c->p.model == m && c->p.k == kk) return prepare_big_impl<T>(c, Q, qu, qi, s);
  FIA_BIG_CASES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t check_cover(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, int32_t* flag, hipStream_t s) {
  if (!c->subset || Q <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_check_cover, dim3(grid_cap((Q + 255) / 256, 4096)), dim3(256), 0, s, Q, qu, qi, c->p.U,
                     c->p.I, c->slot[0].as<int32_t>(), c->slot[1].as<int32_t>(), flag);
  return hipGetLastError();
}

hipError_t query_big(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                     int64_t max_chunks, int32_t* rel_idx, double* influence, double* x_out, int K,
                     int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s, const double* x_in) {
#define X(m, kk, T)                                                                                            \
  if (c->p.model == m && c->p.k == kk)                                                                         \
    return query_big_impl<T>(c, Q, qu, qi, offsets, max_chunks, rel_idx, influence, x_out, K, topk_pos, topk_idx, \
                             topk_val, s, x_in);
  FIA_BIG_CASES(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace fia

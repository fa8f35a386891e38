// MFMA GEMM with fused epilogue, and implicit-GEMM NHWC Conv2d, for gfx950.
//
//   C[m, n] = act(sum_k A[m, k] * W[n, k] + bias[n]) + R[m, n]
//
// Both operands are K-contiguous (activations [M, K] token-major, nn.Linear weights
// [N, K]), which is exactly the MFMA operand layout: lane l of a 16x16x32 bf16 MFMA
// holds 8 consecutive k of row (l & 15), so every fragment read is one 16-byte LDS
// read and every global load is a 16-byte vector.
//
// Tile: BM x BN x BK (BK = 64 bf16 / 32 f32), 256 threads = 4 waves arranged 2 x 2, each
// wave owning a (BM/2) x (BN/2) sub-tile of 16x16 MFMA blocks.  LDS is double-buffered;
// the next K-tile is fetched into registers while the MFMAs of the current one run (one
// __syncthreads per K-step).  LDS rows are padded by 16 bytes: a 16-lane ds_read_b128
// group then touches 16 distinct 4-bank slots (row stride 144 B).
//
// Epilogue: bias + activation are applied in registers, the f32 tile is staged through
// LDS (reusing the operand buffers), and written back as 16-byte row chunks with the
// residual read the same way — the MFMA C layout would otherwise scatter 2-byte stores.
//
// Workgroup -> tile mapping is XCD-aware: the hardware deals consecutive workgroups
// round-robin over the 8 XCDs, so the 1-D grid is remapped so that each XCD receives a
// contiguous run of tiles (n fastest), i.e. the tiles sharing an A row-panel share an L2.
//
// dtype f32 uses v_mfma_f32_16x16x4_f32 (exact f32 products, the parity path): the
// 8 k a lane holds for one 32-deep step are consumed by 8 MFMAs, MFMA s using element s
// of every lane group — a permutation of the k order inside the step, which leaves the
// dot product mathematically unchanged.
//
// ASRC = 1 turns the A loader into an im2col gather from an NHWC map (implicit-GEMM
// convolution, weights packed [Cout][kh][kw][Cin] so that k = (i*kw + j)*Cin + ci).
#include "svk_common.h"
#include "gemm_args.h"
#include <stdio.h>

namespace svk {

constexpr int NTHREADS = 256;


template <typename T> struct Chunk { T v[8]; };

template <typename T>
__device__ __forceinline__ void load_vec8(const T* p, Chunk<T>& c) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(c.v) = *reinterpret_cast<const uint4*>(p);
  } else {
    reinterpret_cast<uint4*>(c.v)[0] = reinterpret_cast<const uint4*>(p)[0];
    reinterpret_cast<uint4*>(c.v)[1] = reinterpret_cast<const uint4*>(p)[1];
  }
}
template <typename T>
__device__ __forceinline__ void zero8(Chunk<T>& c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) c.v[j] = from_f<T>(0.f);
}
template <typename T>
__device__ __forceinline__ void store8(T* dst, const Chunk<T>& c) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(c.v);
  } else {
    reinterpret_cast<uint4*>(dst)[0] = reinterpret_cast<const uint4*>(c.v)[0];
    reinterpret_cast<uint4*>(dst)[1] = reinterpret_cast<const uint4*>(c.v)[1];
  }
}

// All loaders are branch-free: the address is clamped into the valid range, the load is issued
// unconditionally and out-of-range elements are zeroed by a select.  (A conditional load makes
// hipcc branch around it and wait vmcnt(0) per load, serialising the whole K-loop prefetch.)
// The zeroing select is applied when the chunk is written to LDS (after the K-step's MFMAs),
// never right after the load, so that the loads stay in flight across the MFMAs.
// `mask` bit e set = element e valid.
template <typename T, bool VEC>
__device__ __forceinline__ void apply_mask8(Chunk<T>& c, unsigned mask) {
  if constexpr (VEC) {   // all-or-nothing chunks
    uint32_t* w = reinterpret_cast<uint32_t*>(c.v);
#pragma unroll
    for (int j = 0; j < (int)(8 * sizeof(T) / 4); ++j) w[j] = mask ? w[j] : 0u;
  } else if constexpr (sizeof(T) == 2) {
    uint32_t* w = reinterpret_cast<uint32_t*>(c.v);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t keep = ((mask >> (2 * j)) & 1 ? 0x0000FFFFu : 0u) | ((mask >> (2 * j + 1)) & 1 ? 0xFFFF0000u : 0u);
      w[j] &= keep;
    }
  } else {
    uint32_t* w = reinterpret_cast<uint32_t*>(c.v);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = (mask >> j) & 1 ? w[j] : 0u;
  }
}

// Dense row loader: 8 elements of row `row` starting at column k (zero outside [0,rows)x[0,K)).
// VEC requires K % 8 == 0 and 16-byte aligned rows.  Returns the validity mask.
template <typename T, bool VEC>
__device__ __forceinline__ unsigned load_dense(const T* base, long ld, int row, int rows, int k, int K, Chunk<T>& c) {
  const int rc = row < rows ? row : rows - 1;
  if (VEC) {
    const int kc = k < K ? k : ((K - 1) & ~7);   // aligned clamp (rows may be zero-padded past K)
    load_vec8(base + (long)rc * ld + kc, c);
    return (row < rows && k < K) ? 0xFFu : 0u;
  }
  const T* p = base + (long)rc * ld;
  unsigned m = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int kk = k + j;
    c.v[j] = p[kk < K ? kk : K - 1];
    m |= (row < rows && kk < K) ? (1u << j) : 0u;
  }
  return m;
}

struct ConvRow { long base; int iy0, ix0; bool valid; };

template <typename T, bool VEC>
__device__ __forceinline__ unsigned load_im2col(const T* X, const GemmArgs& p, const ConvRow& r, int k, Chunk<T>& c) {
  if (VEC) {  // Cin % 8 == 0: the 8 k of a chunk share one tap
    const int kc = k < p.K ? k : p.K - 8;
    const int tap = kc / p.Cin, ci = kc - tap * p.Cin;
    const int i = tap / p.kw, j = tap - i * p.kw;
    const int iy = r.iy0 + i, ix = r.ix0 + j;
    const bool ok = r.valid && k < p.K && iy >= 0 && iy < p.H && ix >= 0 && ix < p.Wd;
    const int iyc = min(max(iy, 0), p.H - 1), ixc = min(max(ix, 0), p.Wd - 1);
    load_vec8(X + r.base + ((long)iyc * p.Wd + ixc) * p.Cin + ci, c);
    return ok ? 0xFFu : 0u;
  }
  unsigned m = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kk = k + e;
    const int kc = kk < p.K ? kk : p.K - 1;
    const int tap = kc / p.Cin, ci = kc - tap * p.Cin;
    const int i = tap / p.kw, j = tap - i * p.kw;
    const int iy = r.iy0 + i, ix = r.ix0 + j;
    const bool ok = r.valid && kk < p.K && iy >= 0 && iy < p.H && ix >= 0 && ix < p.Wd;
    const int iyc = min(max(iy, 0), p.H - 1), ixc = min(max(ix, 0), p.Wd - 1);
    c.v[e] = X[r.base + ((long)iyc * p.Wd + ixc) * p.Cin + ci];
    m |= ok ? (1u << e) : 0u;
  }
  return m;
}

// Transposed-conv gather for the data gradient of a strided conv: A[m = (b, iy, ix)][k = (i, j, co)]
// = dY[b, (iy + pad - i) / s, (ix + pad - j) / s, co] when both divisions are exact and in range.
// r.iy0 / r.ix0 hold iy + pad / ix + pad.  Stride must be a power of two (sshift).
template <typename T, bool VEC>
__device__ __forceinline__ unsigned load_col2im(const T* X, const GemmArgs& p, const ConvRow& r, int k, Chunk<T>& c) {
  const int smask = (1 << p.sshift) - 1;
  if (VEC) {
    const int kc = k < p.K ? k : p.K - 8;
    const int tap = kc / p.Cin, ci = kc - tap * p.Cin;
    const int i = tap / p.kw, j = tap - i * p.kw;
    const int ny = r.iy0 - i, nx = r.ix0 - j;
    const int oy = max(ny, 0) >> p.sshift, ox = max(nx, 0) >> p.sshift;
    const bool ok = r.valid && k < p.K && ny >= 0 && nx >= 0 && !(ny & smask) && !(nx & smask) && oy < p.H && ox < p.Wd;
    const int oyc = min(oy, p.H - 1), oxc = min(ox, p.Wd - 1);
    load_vec8(X + r.base + ((long)oyc * p.Wd + oxc) * p.Cin + ci, c);
    return ok ? 0xFFu : 0u;
  }
  unsigned m = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kk = k + e;
    const int kc = kk < p.K ? kk : p.K - 1;
    const int tap = kc / p.Cin, ci = kc - tap * p.Cin;
    const int i = tap / p.kw, j = tap - i * p.kw;
    const int ny = r.iy0 - i, nx = r.ix0 - j;
    const int oy = max(ny, 0) >> p.sshift, ox = max(nx, 0) >> p.sshift;
    const bool ok = r.valid && kk < p.K && ny >= 0 && nx >= 0 && !(ny & smask) && !(nx & smask) && oy < p.H && ox < p.Wd;
    const int oyc = min(oy, p.H - 1), oxc = min(ox, p.Wd - 1);
    c.v[e] = X[r.base + ((long)oyc * p.Wd + oxc) * p.Cin + ci];
    m |= ok ? (1u << e) : 0u;
  }
  return m;
}

template <typename T>
__device__ __forceinline__ void mfma_step(const Chunk<T>& a, const Chunk<T>& b, f32x4& acc) {
  if constexpr (sizeof(T) == 2) {
    acc = mfma16x16x32(*reinterpret_cast<const v8_t<T>*>(a.v), *reinterpret_cast<const v8_t<T>*>(b.v), acc);
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[s], b.v[s], acc, 0, 0, 0);
  }
}

// Bijective XCD remap of a 1-D grid (cdna_hip_programming.md §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <typename T> constexpr int bk_of() { return sizeof(T) == 2 ? 64 : 32; }

template <typename T, int BM, int BN>
constexpr int smem_bytes() {
  constexpr int BK = bk_of<T>(), LDK = BK + 16 / (int)sizeof(T);
  constexpr int main_b = 2 * (BM + BN) * LDK * (int)sizeof(T);
  constexpr int epi_b = BM * (BN + 4) * 4;
  return main_b > epi_b ? main_b : epi_b;
}

template <typename T, int BM, int BN, bool VEC, int ASRC, bool EXT>
__global__ __launch_bounds__(NTHREADS) void gemm_kernel(GemmArgs p) {
  constexpr int BK = bk_of<T>();
  constexpr int LDK = BK + 16 / sizeof(T);
  constexpr int CPR = BK / 8;                       // 8-element chunks per tile row
  constexpr int RPP = NTHREADS / CPR;               // rows covered per loader pass
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ACH = BM / RPP, BCH = BN / RPP;     // loader chunks per thread
  constexpr int LDC = BN + 4;                       // f32 epilogue tile row stride
  static_assert(ACH >= 1 && BCH >= 1, "tile too small");

  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<T, BM, BN>()];
  T (*sA)[BM][LDK] = reinterpret_cast<T (*)[BM][LDK]>(smem);
  T (*sB)[BN][LDK] = reinterpret_cast<T (*)[BN][LDK]>(smem + 2 * BM * LDK * sizeof(T));
  float (*sC)[LDC] = reinterpret_cast<float (*)[LDC]>(smem);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = (p.N + BN - 1) / BN;
  const int ntm = (p.M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const T* A = static_cast<const T*>(p.A);
  const T* Wt = static_cast<const T*>(p.W);

  const int lrow = tid / CPR, lk = (tid % CPR) * 8;
  ConvRow crow[ACH];
  if constexpr (ASRC != 0) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int m = m0 + lrow + RPP * i;
      crow[i].valid = m < p.M;
      int mm = crow[i].valid ? m : 0;
      int hw = p.OH * p.OW;
      int b = mm / hw, rem = mm - b * hw;
      int oy = rem / p.OW, ox = rem - oy * p.OW;
      crow[i].base = (long)b * p.H * p.Wd * p.Cin;
      if constexpr (ASRC == 1) {
        crow[i].iy0 = oy * p.stride - p.pad;
        crow[i].ix0 = ox * p.stride - p.pad;
      } else {
        crow[i].iy0 = oy + p.pad;
        crow[i].ix0 = ox + p.pad;
      }
    }
  }

  Chunk<T> ra[ACH], rb[BCH];
  unsigned ma[ACH], mb[BCH];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      if constexpr (ASRC == 1) ma[i] = load_im2col<T, VEC>(A, p, crow[i], k0 + lk, ra[i]);
      else if constexpr (ASRC == 2) ma[i] = load_col2im<T, VEC>(A, p, crow[i], k0 + lk, ra[i]);
      else ma[i] = load_dense<T, VEC>(A, p.lda, m0 + lrow + RPP * i, p.M, k0 + lk, p.K, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) mb[i] = load_dense<T, VEC>(Wt, p.ldw, n0 + lrow + RPP * i, p.N, k0 + lk, p.K, rb[i]);
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) { apply_mask8<T, VEC>(ra[i], ma[i]); store8(&sA[buf][lrow + RPP * i][lk], ra[i]); }
#pragma unroll
    for (int i = 0; i < BCH; ++i) { apply_mask8<T, VEC>(rb[i], mb[i]); store8(&sB[buf][lrow + RPP * i][lk], rb[i]); }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  fetch(0);
  stash(0);
  __syncthreads();

  const int fr = lane & 15, fk = (lane >> 4) * 8;
  auto compute = [&](int buf) {
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      Chunk<T> fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const Chunk<T>*>(&sA[buf][wm * WM + i * 16 + fr][ks * 32 + fk]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const Chunk<T>*>(&sB[buf][wn * WN + j * 16 + fr][ks * 32 + fk]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma_step<T>(fa[i], fb[j], acc[i][j]);
    }
  };
  // steady state: prefetch K-step kt+1 into registers while the MFMAs of kt run; the last step is
  // peeled (no dead prefetch / stash / barrier on the critical path — K = 64 GEMMs have one step)
  for (int kt = 0; kt < nk - 1; ++kt) {
    const int buf = kt & 1;
    fetch((kt + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of this step's MFMAs
    compute(buf);
    stash(buf ^ 1);
    __syncthreads();
  }
  compute((nk - 1) & 1);
  __syncthreads();                       // sC (epilogue) aliases the operand buffers

  if constexpr (!EXT) {
    // Plain epilogue (bias + act + residual).  Part 1: bias + activation in registers, f32 tile -> LDS.
    // C/D map of the 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + r.
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = wn * WN + j * 16 + fr;
      const int n = n0 + cl;
      const float bn = (p.bias && n < p.N) ? p.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sC[wm * WM + i * 16 + (lane >> 4) * 4 + r][cl] = apply_act(acc[i][j][r] + bn, p.act);
    }
    __syncthreads();
    // Part 2: 8-column row chunks, residual added in f32, 16-byte stores.
    T* C = static_cast<T*>(p.C);
    const T* R = static_cast<const T*>(p.R);
    constexpr int CH = BN / 8;
#pragma unroll
    for (int it = 0; it < (BM * CH) / NTHREADS; ++it) {
      const int cidx = tid + it * NTHREADS;
      const int row = cidx / CH, c8 = (cidx % CH) * 8;
      const int m = m0 + row, n = n0 + c8;
      if (m >= p.M || n >= p.N) continue;
      float v[8];
      *reinterpret_cast<float4*>(&v[0]) = *reinterpret_cast<const float4*>(&sC[row][c8]);
      *reinterpret_cast<float4*>(&v[4]) = *reinterpret_cast<const float4*>(&sC[row][c8 + 4]);
      if (p.vec_out && n + 8 <= p.N) {
        if (R) {
          Chunk<T> rr;
          load_vec8(R + (long)m * p.ldr + n, rr);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += to_f(rr.v[e]);
        }
        Chunk<T> o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o.v[e] = from_f<T>(v[e]);
        store8(C + (long)m * p.ldc + n, o);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (n + e >= p.N) break;
          float x = v[e];
          if (R) x += to_f(R[(long)m * p.ldr + n + e]);
          C[(long)m * p.ldc + n + e] = from_f<T>(x);
        }
      }
    }
  } else {
    // Extended epilogue: + row scale (stochastic depth), activation backward (U), unpatchify store.
  T* C = static_cast<T*>(p.C);
  const T* R = static_cast<const T*>(p.R);
  const T* U = static_cast<const T*>(p.U);
  constexpr int CH = BN / 8;
  constexpr int EPI = (BM * CH) / NTHREADS;
  auto out_off = [&](int m, int n) -> long {
    if (p.out_mode == 1) {
      const int PW = p.uW / p.us, PH = p.uH / p.us;
      const int px = m % PW, t = m / PW, py = t % PH, b = t / PH;
      const int ci = n % p.uC, ij = n / p.uC, j = ij % p.us, i = ij / p.us;
      return (((long)b * p.uH + py * p.us + i) * p.uW + px * p.us + j) * p.uC + ci;
    }
    return -1;
  };
  // Part 1: bias + activation in registers, f32 tile -> LDS.
  // C/D map of the 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + r.
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = wn * WN + j * 16 + fr;
    const int n = n0 + cl;
    const float bn = (p.bias && n < p.N) ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sC[wm * WM + i * 16 + (lane >> 4) * 4 + r][cl] = apply_act(acc[i][j][r] + bn, p.act);
  }
  // Prefetch (after the accumulators are dead, so the register peak does not grow): the global loads
  // of the residual R and the activation-backward source U overlap the barrier and the LDS reads.
  Chunk<T> pu[EPI], pr[EPI];
  if (p.vec_out && p.N >= 8) {
#pragma unroll
    for (int it = 0; it < EPI; ++it) {
      const int cidx = tid + it * NTHREADS;
      const int mc = min(m0 + cidx / CH, p.M - 1), nc = min(n0 + (cidx % CH) * 8, p.N - 8);
      if (U) load_vec8(U + (long)mc * p.ldu + nc, pu[it]);
      if (R) {
        const long o = out_off(mc, nc);
        load_vec8(R + (o >= 0 ? o : (long)mc * p.ldr + nc), pr[it]);
      }
    }
  }

  __syncthreads();

  // Part 2: 8-column row chunks, row scale / activation backward / residual in f32, 16-byte stores.
#pragma unroll
  for (int it = 0; it < EPI; ++it) {
    const int cidx = tid + it * NTHREADS;
    const int row = cidx / CH, c8 = (cidx % CH) * 8;
    const int m = m0 + row, n = n0 + c8;
    if (m >= p.M || n >= p.N) continue;
    float v[8];
    *reinterpret_cast<float4*>(&v[0]) = *reinterpret_cast<const float4*>(&sC[row][c8]);
    *reinterpret_cast<float4*>(&v[4]) = *reinterpret_cast<const float4*>(&sC[row][c8 + 4]);
    if (p.rscale) {
      const float sc = p.rscale[m / p.rdiv];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= sc;
    }
    const long om = out_off(m, n);
    const long coff = om >= 0 ? om : (long)m * p.ldc + n, roff = om >= 0 ? om : (long)m * p.ldr + n;
    if (p.vec_out && n + 8 <= p.N) {
      if (U) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= act_grad(to_f(pu[it].v[e]), p.uact);
      }
      if (R) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += to_f(pr[it].v[e]);
      }
      Chunk<T> o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o.v[e] = from_f<T>(v[e]);
      store8(C + coff, o);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (n + e >= p.N) break;
        float x = v[e];
        if (U) x *= act_grad(to_f(U[(long)m * p.ldu + n + e]), p.uact);
        if (R) x += to_f(R[roff + e]);
        C[coff + e] = from_f<T>(x);
      }
    }
  }
  }
}

static bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

// f32 GEMMs with few rows (the train step's f32 classifier heads and their gradients: M = 88 frames,
// K = 512 - 2048): the 64 x 64 register-staged tiles give 16 workgroups on 256 CUs (1-7 TF/s).  Here a
// workgroup owns 16 x 16 outputs and its four waves split K (lane: one row, 4 consecutive columns, 16-byte
// loads along k when aligned); the partial sums meet in LDS and one thread per output runs the same epilogue
// as gemm_kernel (act(acc + bias), row scale, activation backward, residual).
template <bool VK>
__global__ __launch_bounds__(256) void gemm_f32_smallm(GemmArgs p) {
  __shared__ float red[4][16][17];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tn = (p.N + 15) / 16;
  const int m0 = (blockIdx.x / tn) * 16, n0 = (blockIdx.x % tn) * 16;
  const int mi = lane & 15, nj = (lane >> 4) * 4;
  const float* A = static_cast<const float*>(p.A) + (long)min(m0 + mi, p.M - 1) * p.lda;
  const float* Wr[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) Wr[j] = static_cast<const float*>(p.W) + (long)min(n0 + nj + j, p.N - 1) * p.ldw;
  const int chunk = ((p.K + 15) / 16) * 4;            // per wave, a multiple of 4
  const int k0 = w * chunk, k1 = min(k0 + chunk, p.K);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int k = k0;
  if constexpr (VK) {
    for (; k + 4 <= k1; k += 4) {
      const float4 a = *reinterpret_cast<const float4*>(A + k);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 b = *reinterpret_cast<const float4*>(Wr[j] + k);
        acc[j] = fmaf(a.x, b.x, acc[j]);
        acc[j] = fmaf(a.y, b.y, acc[j]);
        acc[j] = fmaf(a.z, b.z, acc[j]);
        acc[j] = fmaf(a.w, b.w, acc[j]);
      }
    }
  }
  for (; k < k1; ++k) {
    const float a = A[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = fmaf(a, Wr[j][k], acc[j]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w][mi][nj + j] = acc[j];
  __syncthreads();
  const int row = tid >> 4, col = tid & 15, m = m0 + row, n = n0 + col;
  if (m >= p.M || n >= p.N) return;
  float v = red[0][row][col] + red[1][row][col] + red[2][row][col] + red[3][row][col];
  v = apply_act(v + (p.bias ? p.bias[n] : 0.f), p.act);
  if (p.rscale) v *= p.rscale[m / p.rdiv];
  if (p.U) v *= act_grad(static_cast<const float*>(p.U)[(long)m * p.ldu + n], p.uact);
  if (p.R) v += static_cast<const float*>(p.R)[(long)m * p.ldr + n];
  static_cast<float*>(p.C)[(long)m * p.ldc + n] = v;
}

template <typename T, int ASRC>
static int launch_gemm(GemmArgs a, bool vec, hipStream_t st) {
  const int M = a.M, N = a.N;
  const long vw = 16 / (long)sizeof(T);
  a.vec_out = aligned16(a.C) && (a.ldc % vw == 0) && (!a.R || (aligned16(a.R) && a.ldr % vw == 0)) &&
              (!a.U || (aligned16(a.U) && a.ldu % vw == 0)) && (a.out_mode == 0 || a.uC % 8 == 0);
  const bool ext = a.rscale || a.U || a.out_mode;
  set_pk_reject(vec ? "" : "unaligned/K%8");
  if constexpr (sizeof(T) == 2 && ASRC <= 1) {
    if (vec && gemm_pk_try<T>(a, st, ASRC) == 0) return SVK_OK;
  } else {
    set_pk_reject(sizeof(T) == 2 ? "asrc" : "f32");
  }
  if constexpr (sizeof(T) == 4 && ASRC == 0) {
    // few rows, long K: the 64 x 64 tiles would leave most CUs idle
    const long tiles64 = (long)((M + 63) / 64) * ((N + 63) / 64);
    static const bool smallm_on = !getenv("SVK_NO_F32_SMALLM");
    // (N >= 256: the classifier heads; narrower few-row GEMMs — e.g. a short video's MS-TCN input layer — keep
    // gemm_kernel's summation order, so a video's rows come out the same alone and in a ragged batch)
    if (smallm_on && a.out_mode == 0 && M <= 256 && a.N >= 256 && a.K >= 128 && tiles64 < 128) {
      const bool vk = aligned16(a.A) && aligned16(a.W) && a.lda % 4 == 0 && a.ldw % 4 == 0;
      const dim3 grid((unsigned)(((M + 15) / 16) * ((N + 15) / 16)));
      if (vk) hipLaunchKernelGGL(gemm_f32_smallm<true>, grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL(gemm_f32_smallm<false>, grid, dim3(256), 0, st, a);
      set_last_kernel(vk ? "gemm_f32_smallm<true>" : "gemm_f32_smallm<false>");
      return check_launch("gemm_f32_smallm");
    }
  }
  auto go = [&](auto bm_c, auto bn_c) {
    constexpr int BM = decltype(bm_c)::value, BN = decltype(bn_c)::value;
    const long nwg = (long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    dim3 grid((unsigned)nwg);
    static char names[2][2][96];
    char* nm = names[vec][ext];
    if (!nm[0])
      snprintf(nm, 96, "gemm_kernel<%s, %d, %d, %s, %d, %s>", type_name<T>(), BM, BN,
               vec ? "true" : "false", ASRC, ext ? "true" : "false");
    static thread_local char full[160];
    snprintf(full, sizeof(full), "%s [%s]", nm, pk_reject());
    set_last_kernel(full);
    if (ext) {
      if (vec) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, true, ASRC, true>), grid, dim3(NTHREADS), 0, st, a);
      else hipLaunchKernelGGL((gemm_kernel<T, BM, BN, false, ASRC, true>), grid, dim3(NTHREADS), 0, st, a);
    } else {
      if (vec) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, true, ASRC, false>), grid, dim3(NTHREADS), 0, st, a);
      else hipLaunchKernelGGL((gemm_kernel<T, BM, BN, false, ASRC, false>), grid, dim3(NTHREADS), 0, st, a);
    }
  };
  using I64 = std::integral_constant<int, 64>;
  using I128 = std::integral_constant<int, 128>;
  if (N <= 64) {
    if ((long)((M + 127) / 128) >= 512) go(I128{}, I64{}); else go(I64{}, I64{});
  } else {
    long tiles128 = (long)((M + 127) / 128) * ((N + 127) / 128);
    if (tiles128 >= 512) go(I128{}, I128{}); else go(I64{}, I64{});
  }
  return check_launch("gemm");
}


// ---- weight gradient: dW[n][k] += sum_m dY[m][n] * X[m][k] ------------------------------------
// Both operands arrive m-major (token rows), but the MFMA wants the reduction index m contiguous
// per lane, so each 32-row slab of dY and X is staged TRANSPOSED in LDS ([n][m] / [k][m]); the
// fragment reads are then the same 16-byte reads as the forward GEMM.  Loader mapping: thread ->
// (m = tid & 31, 8-column chunk = tid >> 5), which makes the transposed 2/4-byte LDS writes
// conflict-free (32 consecutive m per column).  Tile 64 (n) x 64 (k); the M range is split over
// gridDim.y workgroups whose partial tiles are f32-atomically added into dW.
// BSRC = 1: X is an NHWC map read through the conv im2col gather (conv weight gradient, dW packed
// [Cout][kh][kw][Cin] like the forward weights).
struct WgradArgs {
  const void* dY; long ldy;
  const void* X; long ldx;
  float* dW; long lddw;
  int M, N, K, mchunk;
  int H, Wd, Cin, OH, OW, kw, stride, pad;
  // batching over gridDim.z: z -> (z / nzi, z % nzi) outer/inner offsets (elements)
  int nzi;
  long sa_o, sa_i, sx_o, sx_i, sw_o, sw_i;
  float* db;            // optional bias gradient db[n] += sum_m dY[m, n] (first K-tile column only)
};

template <typename T, bool VECA, bool VECB, int BSRC>
__global__ __launch_bounds__(NTHREADS) void wgrad_kernel(WgradArgs p) {
  constexpr int LDT = 32 + 16 / (int)sizeof(T);   // 40 bf16 (80 B rows) / 36 f32 (144 B rows)
  __shared__ __attribute__((aligned(16))) T sA[2][64][LDT];
  __shared__ __attribute__((aligned(16))) T sB[2][64][LDT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int ntk = (p.K + 63) / 64;
  const int n0 = (blockIdx.x / ntk) * 64, k0 = (blockIdx.x % ntk) * 64;
  const int mbeg = blockIdx.y * p.mchunk;
  const int mend = min(mbeg + p.mchunk, p.M);
  const int zo = blockIdx.z / p.nzi, zi = blockIdx.z - (blockIdx.z / p.nzi) * p.nzi;
  const T* dY = static_cast<const T*>(p.dY) + zo * p.sa_o + zi * p.sa_i;
  const T* X = static_cast<const T*>(p.X) + zo * p.sx_o + zi * p.sx_i;
  float* dWz = p.dW + zo * p.sw_o + zi * p.sw_i;
  const int lm = tid & 31, lc = (tid >> 5) * 8;

  Chunk<T> ra, rb;
  unsigned ma, mb;
  GemmArgs ga{};   // geometry for the im2col loader
  if constexpr (BSRC == 1) {
    ga.K = p.K; ga.H = p.H; ga.Wd = p.Wd; ga.Cin = p.Cin; ga.OH = p.OH; ga.OW = p.OW; ga.kw = p.kw;
    ga.stride = p.stride; ga.pad = p.pad;
  }
  auto fetch = [&](int m0) {
    const int m = m0 + lm;
    const bool mv = m < mend;
    ma = load_dense<T, VECA>(dY, p.ldy, mv ? m : p.M, p.M, n0 + lc, p.N, ra);   // rows >= M are masked
    if constexpr (BSRC == 1) {
      ConvRow r;
      r.valid = mv;
      const int mm = mv ? m : 0;
      const int hw = p.OH * p.OW;
      const int b = mm / hw, rem = mm - b * hw;
      const int oy = rem / p.OW, ox = rem - oy * p.OW;
      r.base = (long)b * p.H * p.Wd * p.Cin;
      r.iy0 = oy * p.stride - p.pad;
      r.ix0 = ox * p.stride - p.pad;
      mb = load_im2col<T, VECB>(X, ga, r, k0 + lc, rb);
    } else {
      mb = load_dense<T, VECB>(X, p.ldx, mv ? m : p.M, p.M, k0 + lc, p.K, rb);
    }
  };
  const bool do_db = p.db != nullptr && (blockIdx.x % ntk) == 0;
  float dsum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) dsum[e] = 0.f;
  auto stash = [&](int buf) {
    apply_mask8<T, VECA>(ra, ma);
    apply_mask8<T, VECB>(rb, mb);
    if (do_db) {
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum[e] += to_f(ra.v[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sA[buf][lc + e][lm] = ra.v[e];
      sB[buf][lc + e][lm] = rb.v[e];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = (lane >> 4) * 8;
  fetch(mbeg);
  stash(0);
  __syncthreads();
  int buf = 0;
  for (int m0 = mbeg; m0 < mend; m0 += 32) {
    fetch(m0 + 32);
    __builtin_amdgcn_sched_barrier(0);
    Chunk<T> fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const Chunk<T>*>(&sA[buf][wn * 32 + i * 16 + fr][fk]);
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = *reinterpret_cast<const Chunk<T>*>(&sB[buf][wk * 32 + j * 16 + fr][fk]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) mfma_step<T>(fa[i], fb[j], acc[i][j]);
    stash(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  if (do_db) {
    // the stash after the last step loaded a fully masked slab, so dsum holds exactly this WG's rows
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = dsum[e];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
      dsum[e] = v;
    }
    if ((tid & 31) == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (n0 + lc + e < p.N) atomicAdd(p.db + n0 + lc + e, dsum[e]);
    }
  }
  // C map: col (k) = lane & 15, row (n) = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = k0 + wk * 32 + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (n < p.N && k < p.K) atomicAdd(dWz + (long)n * p.lddw + k, acc[i][j][r]);
      }
    }
}

template <typename T, int BSRC>
static int launch_wgrad(WgradArgs a, bool veca, bool vecb, hipStream_t st, int Z = 1) {
  if (a.nzi <= 0) a.nzi = 1;
  const long tiles = (long)((a.N + 63) / 64) * ((a.K + 63) / 64);
  // split M so that the grid holds ~1024 workgroups, each with >= 1024 rows (fewer, longer
  // workgroups: the partial tiles and bias sums are f32 atomics on few addresses)
  long splits = std::max<long>(1, std::min<long>((1024 + tiles * Z - 1) / (tiles * Z), (a.M + 1023) / 1024));
  long chunk = (a.M + splits - 1) / splits;
  chunk = (chunk + 31) / 32 * 32;
  splits = (a.M + chunk - 1) / chunk;
  a.mchunk = (int)chunk;
  dim3 grid((unsigned)tiles, (unsigned)splits, (unsigned)Z);
  if (veca && vecb) hipLaunchKernelGGL((wgrad_kernel<T, true, true, BSRC>), grid, dim3(NTHREADS), 0, st, a);
  else if (veca) hipLaunchKernelGGL((wgrad_kernel<T, true, false, BSRC>), grid, dim3(NTHREADS), 0, st, a);
  else if (vecb) hipLaunchKernelGGL((wgrad_kernel<T, false, true, BSRC>), grid, dim3(NTHREADS), 0, st, a);
  else hipLaunchKernelGGL((wgrad_kernel<T, false, false, BSRC>), grid, dim3(NTHREADS), 0, st, a);
  return check_launch("wgrad");
}

}  // namespace svk

using namespace svk;

extern "C" int svk_gemm_ex(int dtype, const void* A, long lda, const void* W, long ldw, const float* bias,
                           const float* row_scale, int rows_per_scale, const void* U, long ldu, int uact,
                           const void* R, long ldr, void* C, long ldc, int M, int N, int K, int act, void* stream) {
  if (M < 0 || N <= 0 || K <= 0 || !A || !W || !C || (row_scale && rows_per_scale <= 0)) {
    set_error("svk_gemm: bad args M=%d N=%d K=%d", M, N, K); return SVK_EINVAL;
  }
  if (M == 0) return SVK_OK;
  if (lda < K || ldw < K || ldc < N || (R && ldr < N)) { set_error("svk_gemm: leading dims too small"); return SVK_EINVAL; }
  GemmArgs a{};
  a.A = A; a.lda = lda; a.W = W; a.ldw = ldw; a.bias = bias; a.R = R; a.ldr = ldr; a.C = C; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K; a.act = act; a.rscale = row_scale; a.rdiv = rows_per_scale;
  if (U && ldu < N) { set_error("svk_gemm: ldu too small"); return SVK_EINVAL; }
  a.U = U; a.ldu = ldu; a.uact = uact;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    const long vecw = 16 / (long)sizeof(T);
    bool vec = aligned16(A) && aligned16(W) && (lda % vecw == 0) && (ldw % vecw == 0) && (K % 8 == 0);
    return launch_gemm<T, 0>(a, vec, st);
  });
}

extern "C" int svk_gemm(int dtype, const void* A, long lda, const void* W, long ldw, const float* bias,
                        const void* R, long ldr, void* C, long ldc, int M, int N, int K, int act, void* stream) {
  return svk_gemm_ex(dtype, A, lda, W, ldw, bias, nullptr, 1, nullptr, 0, 0, R, ldr, C, ldc, M, N, K, act, stream);
}

extern "C" int svk_gemm_unpatchify(int dtype, const void* A, long lda, const void* W, long ldw, const void* R,
                                   void* Y, int B, int H, int Wd, int s, int C, int K, void* stream) {
  if (B < 0 || H <= 0 || Wd <= 0 || s <= 0 || C <= 0 || K <= 0 || H % s || Wd % s || !A || !W || !Y || lda < K ||
      ldw < K) {
    set_error("svk_gemm_unpatchify: bad args"); return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  GemmArgs a{};
  a.A = A; a.lda = lda; a.W = W; a.ldw = ldw; a.R = R; a.ldr = 0; a.C = Y; a.ldc = 0;
  a.M = B * (H / s) * (Wd / s); a.N = s * s * C; a.K = K; a.rdiv = 1;
  a.out_mode = 1; a.uH = H; a.uW = Wd; a.us = s; a.uC = C;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    const long vecw = 16 / (long)sizeof(T);
    bool vec = aligned16(A) && aligned16(W) && (lda % vecw == 0) && (ldw % vecw == 0) && (K % 8 == 0);
    return launch_gemm<T, 0>(a, vec, st);
  });
}

extern "C" int svk_conv2d_nhwc(int dtype, const void* X, int B, int H, int W, int Cin, const void* Wt,
                               const float* bias, const void* R, void* Y, int Cout, int k, int stride, int pad,
                               int act, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || k <= 0 || stride <= 0 || pad < 0 || !X || !Wt || !Y) {
    set_error("svk_conv2d_nhwc: bad args"); return SVK_EINVAL;
  }
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  if (OH <= 0 || OW <= 0) { set_error("svk_conv2d_nhwc: empty output"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long M = (long)B * OH * OW;
  if (M > 0x7fffffffL) { set_error("svk_conv2d_nhwc: too many output pixels"); return SVK_EUNSUPPORTED; }
  GemmArgs a{};
  a.A = X; a.lda = 0; a.W = Wt; a.ldw = (long)k * k * Cin; a.bias = bias; a.R = R; a.ldr = Cout; a.C = Y; a.ldc = Cout;
  a.M = (int)M; a.N = Cout; a.K = k * k * Cin; a.act = act;
  a.H = H; a.Wd = W; a.Cin = Cin; a.OH = OH; a.OW = OW; a.kw = k; a.stride = stride; a.pad = pad;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    bool vec = aligned16(X) && aligned16(Wt) && (Cin % 8 == 0);
    return launch_gemm<T, 1>(a, vec, st);
  });
}

// Sequence-reduction conv + LayerNorm (Attention.sr -> Attention.norm, mix_transformer_evp.py:115-117):
// for the long-K patchify convs whose row-tile grid cannot fill the chip, split K into ks parts
// written as f32 slabs and reduce them in the LayerNorm kernel (workspace ks * M * Cout * 4 bytes);
// otherwise the conv writes Y and the LayerNorm runs in place.
static int conv_ln_ksplit(int dtype, long M, int N, int K, int Cin) {
  // measured (B = 256): splitting pays for the N <= 128 stages (64 x 64 tiles, 196 / 392 of them);
  // at N = 320 (490 128 x 64 tiles) the extra slab pass costs more than the occupancy gains
  if ((dtype != SVK_BF16 && dtype != SVK_F16) || K % 64 || Cin % 8 || N % 4 || N > 128) return 1;
  const int nk = K / 64;
  const int bm = splitk_bm();
  const long tiles = ((M + bm - 1) / bm) * ((N + 63) / 64);
  int ks = 1;
  while (tiles * ks < 768 && nk % (2 * ks) == 0 && nk / (2 * ks) >= 4) ks *= 2;
  return ks;
}

extern "C" long svk_conv2d_ln_workspace(int dtype, int B, int H, int W, int Cin, int Cout, int k, int stride, int pad) {
  if (B <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || k <= 0 || stride <= 0 || pad < 0) return 0;
  const long OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  if (OH <= 0 || OW <= 0) return 0;
  const long M = (long)B * OH * OW;
  const int ks = conv_ln_ksplit(dtype, M, Cout, k * k * Cin, Cin);
  return ks > 1 ? (long)ks * M * Cout * 4 : 0;
}

extern "C" int svk_conv2d_ln_nhwc(int dtype, const void* X, int B, int H, int W, int Cin, const void* Wt,
                                  const float* bias, const float* gamma, const float* beta, float eps, void* Y,
                                  int Cout, int k, int stride, int pad, void* ws, long ws_bytes, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || k <= 0 || stride <= 0 || pad < 0 || !X || !Wt || !Y ||
      !bias || !gamma || !beta) {
    set_error("svk_conv2d_ln_nhwc: bad args"); return SVK_EINVAL;
  }
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  if (OH <= 0 || OW <= 0) { set_error("svk_conv2d_ln_nhwc: empty output"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long M = (long)B * OH * OW;
  if (M > 0x7fffffffL) { set_error("svk_conv2d_ln_nhwc: too many output pixels"); return SVK_EUNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  const int ks = conv_ln_ksplit(dtype, M, Cout, k * k * Cin, Cin);
  if (ks > 1 && ws && ws_bytes >= (long)ks * M * Cout * 4) {
    GemmArgs a{};
    a.A = X; a.lda = 0; a.W = Wt; a.ldw = (long)k * k * Cin; a.C = Y; a.ldc = Cout;
    a.M = (int)M; a.N = Cout; a.K = k * k * Cin;
    a.H = H; a.Wd = W; a.Cin = Cin; a.OH = OH; a.OW = OW; a.kw = k; a.stride = stride; a.pad = pad;
    a.ksplit = ks; a.slab = static_cast<float*>(ws);
    SVK_DISPATCH_H16(dtype, T, {
      if (gemm_pk_conv_splitk<T>(a, st) == 0) {
        int rc = check_launch("conv2d_ln splitk");
        if (rc) return rc;
        return splitk_layernorm<T>(a.slab, ks, bias, static_cast<T*>(Y), (int)M, Cout, gamma, beta, eps, st);
      }
    });
  }
  int rc = svk_conv2d_nhwc(dtype, X, B, H, W, Cin, Wt, bias, nullptr, Y, Cout, k, stride, pad, SVK_ACT_NONE, stream);
  if (rc) return rc;
  return svk_layernorm(dtype, Y, Cout, Y, Cout, gamma, beta, (int)M, Cout, eps, stream);
}

extern "C" int svk_conv2d_dgrad_nhwc(int dtype, const void* dY, int B, int OH, int OW, int Cout, const void* Wd,
                                     const void* R, void* dX, int H, int W, int Cin, int k, int stride, int pad,
                                     void* stream) {
  if (B < 0 || OH <= 0 || OW <= 0 || Cout <= 0 || H <= 0 || W <= 0 || Cin <= 0 || k <= 0 || pad < 0 || !dY || !Wd ||
      !dX || stride <= 0 || (stride & (stride - 1))) {
    set_error("svk_conv2d_dgrad_nhwc: bad args (stride must be a power of two)"); return SVK_EINVAL;
  }
  if ((H + 2 * pad - k) / stride + 1 != OH || (W + 2 * pad - k) / stride + 1 != OW) {
    set_error("svk_conv2d_dgrad_nhwc: geometry mismatch"); return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  const long M = (long)B * H * W;
  if (M > 0x7fffffffL) { set_error("svk_conv2d_dgrad_nhwc: too many pixels"); return SVK_EUNSUPPORTED; }
  GemmArgs a{};
  a.A = dY; a.lda = 0; a.W = Wd; a.ldw = (long)k * k * Cout; a.R = R; a.ldr = Cin; a.C = dX; a.ldc = Cin;
  a.M = (int)M; a.N = Cin; a.K = k * k * Cout; a.act = 0; a.rdiv = 1;
  a.H = OH; a.Wd = OW; a.Cin = Cout; a.OH = H; a.OW = W; a.kw = k; a.stride = stride; a.pad = pad;
  a.sshift = __builtin_ctz(stride);
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    bool vec = aligned16(dY) && aligned16(Wd) && (Cout % 8 == 0);
    return launch_gemm<T, 2>(a, vec, st);
  });
}

// Batched weight-gradient reduction used by the attention backward (dK = dS^T Q, dV = P^T dO per
// frame and head).  dY rows may be padded past N (ldy >= N rounded up to 8, zero-filled) which
// allows the vector loader whenever the alignment holds.
int svk::wgrad_batched(int dtype, const void* dY, long ldy, long sa_o, long sa_i, const void* X, long ldx, long sx_o,
                  long sx_i, float* dW, long lddw, long sw_o, long sw_i, int Z, int nzi, int M, int N, int K,
                  hipStream_t st) {
  WgradArgs a{};
  a.dY = dY; a.ldy = ldy; a.X = X; a.ldx = ldx; a.dW = dW; a.lddw = lddw; a.M = M; a.N = N; a.K = K;
  a.nzi = nzi; a.sa_o = sa_o; a.sa_i = sa_i; a.sx_o = sx_o; a.sx_i = sx_i; a.sw_o = sw_o; a.sw_i = sw_i;
  SVK_DISPATCH_DTYPE(dtype, T, {
    if constexpr (sizeof(T) == 2) {
      if (wgrad_pk_try<T>(dY, ldy, sa_o, sa_i, X, ldx, sx_o, sx_i, dW, lddw, sw_o, sw_i, nullptr, Z, nzi, M, N, K,
                          st) == 0)
        return SVK_OK;
    }
    const long vw = 16 / (long)sizeof(T);
    const bool va = aligned16(dY) && ldy % vw == 0 && sa_o % vw == 0 && sa_i % vw == 0 && ldy >= (N + 7) / 8 * 8;
    const bool vb = aligned16(X) && ldx % vw == 0 && sx_o % vw == 0 && sx_i % vw == 0 && K % 8 == 0;
    return launch_wgrad<T, 0>(a, va, vb, st, Z);
  });
}

extern "C" int svk_gemm_wgrad(int dtype, const void* dY, long ldy, const void* X, long ldx, float* dW, long lddw,
                              float* db, int M, int N, int K, void* stream) {
  if (M < 0 || N <= 0 || K <= 0 || !dY || !X || !dW || ldy < N || ldx < K || lddw < K) {
    set_error("svk_gemm_wgrad: bad args"); return SVK_EINVAL;
  }
  if (M == 0) return SVK_OK;
  WgradArgs a{};
  a.dY = dY; a.ldy = ldy; a.X = X; a.ldx = ldx; a.dW = dW; a.lddw = lddw; a.M = M; a.N = N; a.K = K; a.db = db;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    if constexpr (sizeof(T) == 2) {
      if (wgrad_pk_try<T>(dY, ldy, 0, 0, X, ldx, 0, 0, dW, lddw, 0, 0, db, 1, 1, M, N, K, st) == 0) return SVK_OK;
    }
    const long vw = 16 / (long)sizeof(T);
    const bool va = aligned16(dY) && ldy % vw == 0 && N % 8 == 0;
    const bool vb = aligned16(X) && ldx % vw == 0 && K % 8 == 0;
    return launch_wgrad<T, 0>(a, va, vb, st);
  });
}

extern "C" int svk_conv2d_wgrad_nhwc(int dtype, const void* X, int B, int H, int W, int Cin, const void* dY,
                                     int Cout, int k, int stride, int pad, float* dW, float* db, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || k <= 0 || stride <= 0 || pad < 0 || !X || !dY || !dW) {
    set_error("svk_conv2d_wgrad_nhwc: bad args"); return SVK_EINVAL;
  }
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  if (OH <= 0 || OW <= 0) { set_error("svk_conv2d_wgrad_nhwc: empty output"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long M = (long)B * OH * OW;
  if (M > 0x7fffffffL) { set_error("svk_conv2d_wgrad_nhwc: too many pixels"); return SVK_EUNSUPPORTED; }
  WgradArgs a{};
  a.dY = dY; a.ldy = Cout; a.X = X; a.ldx = 0; a.dW = dW; a.lddw = (long)k * k * Cin;
  a.M = (int)M; a.N = Cout; a.K = k * k * Cin; a.db = db;
  a.H = H; a.Wd = W; a.Cin = Cin; a.OH = OH; a.OW = OW; a.kw = k; a.stride = stride; a.pad = pad;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    if constexpr (sizeof(T) == 2) {
      if (wgrad_pk_conv_try<T>(X, B, H, W, Cin, dY, Cout, k, stride, pad, OH, OW, dW, db, st) == 0) return SVK_OK;
    }
    const bool va = aligned16(dY) && Cout % 8 == 0;
    const bool vb = aligned16(X) && Cin % 8 == 0;
    return launch_wgrad<T, 1>(a, va, vb, st);
  });
}

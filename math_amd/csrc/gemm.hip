// fp64 GEMM on the CDNA4 matrix cores (v_mfma_f64_16x16x4_f64).
//
// C = alpha op(A) op(B) + beta C, optionally only the lower triangle of C.
// Used for the dense contractions of multiply (rev/mat/fun/multiply.hpp:65-135)
// and of the blocked Cholesky forward / Murray adjoint
// (rev/mat/fun/cholesky_decompose.hpp:135-158).
//
// Tiling: a 256-thread workgroup (4 waves, 2x2) owns a BM x BN tile of C;
// each wave owns (BM/2) x (BN/2) = TM x TN MFMA tiles of 16x16 held in
// accumulators.  K advances in stages of BK (16 for the 128 x 128 and
// 64 x 64 tiles, 32 for the 32-wide ones) staged through LDS in unpadded,
// XOR-swizzled images (lds_layout): conflict-free ds_read_b64 fragment reads
// (16 consecutive rows/cols x 4 k) and staging stores.
// Global->LDS staging goes through registers (one stage of prefetch for the
// 128 x 128 tile, two for the small tiles) into double-buffered LDS; the
// beta * C operand of the epilogue is fetched before the K loop.
// Split-K writes fixed-order partial slabs reduced by a second kernel, so the
// result is bitwise deterministic run to run.
#include "smg_internal.h"
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#ifndef SMG_GEMM_TRI128_MIN
#define SMG_GEMM_TRI128_MIN 1024  // fewest 128 x 128 tiles a product with a triangular operand takes them at
#endif
#ifndef SMG_GEMM_KS2_MAX
#define SMG_GEMM_KS2_MAX 1536  // largest 64 x 64 tile count that takes the 8-wave variant
#endif
#ifndef SMG_GEMM_NR64
#define SMG_GEMM_NR64 2
#endif
#ifndef SMG_GEMM_NR32
#define SMG_GEMM_NR32 2
#endif

namespace {

// LDS images of the operand tiles, unpadded and XOR-swizzled so that both
// the staging stores (32 consecutive elements along the contiguous dim per
// half-wave) and the MFMA fragment reads (16 consecutive rows x 2 k per
// half-wave, ds_read_b64) hit 32 distinct bank pairs.
template <int BM, int BK, bool KCONTIG>
struct lds_layout;
template <int BM, int BK>
struct lds_layout<BM, BK, false> {  // [k][BM], row index ^ 16 on odd k
  static_assert(BM % 32 == 0, "BM");
  static constexpr int size = BK * BM;
  __device__ static int at(int i, int kk) { return kk * BM + (i ^ ((kk & 1) << 4)); }
};
template <int BM, int BK>
struct lds_layout<BM, BK, true> {  // [BM][BK], k index ^ f(row)
  static_assert(BK == 16 || BK == 32, "BK");
  static constexpr int size = BM * BK;
  __device__ static int at(int i, int kk) {
    return i * BK + (kk ^ (BK == 16 ? (i & 14) : ((i & 15) << 1)));
  }
};

// compile-time unrolled loop: f(std::integral_constant<int, 0>) .. f(<N - 1>)
template <int I, int N, typename F>
__device__ __forceinline__ void smg_static_for_impl(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    smg_static_for_impl<I + 1, N>(f);
  }
}
template <int N, typename F>
__device__ __forceinline__ void smg_static_for(F&& f) {
  smg_static_for_impl<0, N>(f);
}

// every out-of-range operand element is loaded from this zero instead of
// being masked after the load (see load_tile)
__device__ double g_gemm_zero[2] = {0.0, 0.0};  // global (not constant) address space: keeps the operand loads global_load, not flat_load

// Operand X viewed as a (rows x k) matrix in the kernel's orientation:
//   KCONTIG == false : element (i, kk) at X[i + kk*ld]
//   KCONTIG == true  : element (i, kk) at X[kk + i*ld]
// Branch- and select-free on the loaded data: an out-of-range element's
// ADDRESS is redirected to g_gemm_zero, so the loaded register goes straight
// to its LDS store.  (A select on the loaded value lets the scheduler hoist
// the select -- and with it a wait for that load -- ahead of the previous
// stage's MFMAs, which serialises the prefetch.)
template <int BM, int BK, bool KCONTIG, int NT = 256>
__device__ __forceinline__ void load_tile(const double* __restrict__ X, int ld,
                                          int rows, int k, int i0, int k0,
                                          double (&r)[BM * BK / NT]) {
  constexpr int PER = BM * BK / NT;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int e = threadIdx.x + NT * q;
    int i, kk;
    if (KCONTIG) {
      i = e / BK;
      kk = e % BK;
    } else {
      kk = e / BM;
      i = e % BM;
    }
    const int gi = i0 + i, gk = k0 + kk;
    const double* p = KCONTIG ? X + ((size_t)gi * ld + gk) : X + (gi + (size_t)gk * ld);
    r[q] = *((gi < rows && gk < k) ? p : g_gemm_zero);
  }
}

template <int BM, int BK, bool KCONTIG, int NT = 256>
__device__ __forceinline__ void store_tile(double* lds, const double (&r)[BM * BK / NT]) {
  constexpr int PER = BM * BK / NT;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int e = threadIdx.x + NT * q;
    int i, kk;
    if (KCONTIG) {
      i = e / BK;
      kk = e % BK;
    } else {
      kk = e / BM;
      i = e % BM;
    }
    lds[lds_layout<BM, BK, KCONTIG>::at(i, kk)] = r[q];
  }
}

__device__ __forceinline__ void tri_decode(int t, int& bi, int& bj) {
  // t -> (bi, bj) with bj <= bi, row-major over the lower triangle of tiles
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  bi = r;
  bj = t - r * (r + 1) / 2;
}

// t -> (bi, bj) over the lower triangle of T x T tiles in groups of 8 block
// rows, each group column by column (its rows i >= j within a column): the
// tiles in flight at once share a few A row panels and B column panels, where
// the row-major order swept every B panel of a row before the next row
__device__ __forceinline__ void tri_decode_grouped(int t, int T, int& bi, int& bj) {
  constexpr int G = 8;
  int r, c;
  tri_decode(t, r, c);
  const int r0 = r / G * G, r1 = min(r0 + G, T), h = r1 - r0;
  int q = t - r0 * (r0 + 1) / 2;
  if (q < r0 * h) {
    bi = r0 + q % h;
    bj = q / h;
    return;
  }
  q -= r0 * h;
  int j = r0;
  while (q >= r1 - j) {
    q -= r1 - j;
    ++j;
  }
  bi = j + q;
  bj = j;
}

// MODE: 0 = full C, 1 = lower / 2 = upper triangle of C only (BM == BN, m == n),
//   3 = the lower triangle computed and stored mirrored too (a symmetric C
//       from its lower half: no separate sym_from_lower pass),
//   4 = full C plus a second output C2 = tril(C) with halved diagonal (the
//       Murray reverse's D_adj image of its symbolic step: no separate pass).
// Split-K (slab != null): partial tiles into fixed-order slabs, summed by
// k_splitk_reduce (an in-kernel last-workgroup fixup measured slower: the
// tail reduction ran on one CU per tile, 90 -> 172 us for 512 x 2560 x 1536).
// KS: waves per output sub-tile (KS = 2: 8 waves, the two 4-wave groups take
// alternate halves of every K stage and their accumulators are summed in the
// epilogue -- twice the waves per CU for grids that cover the CUs only once
// or twice)
template <int BM, int BN, int BK, bool TA, bool TB, int MODE, int KS = 1>
__global__ __launch_bounds__(256 * KS) void k_gemm(
    int m, int n, int k, double alpha, const double* __restrict__ A, int lda,
    const double* __restrict__ B, int ldb, double beta, double* __restrict__ C,
    int ldc, int tiles_m, int ntiles, int kchunk, double* __restrict__ slab, long long sA,
    long long sB, long long sC, int px, int ntp, int tri, double* __restrict__ C2, int ldc2, int bz) {
  constexpr bool LOWT = MODE == 1 || MODE == 3;  // lower-triangle tiles
  constexpr bool UPT = MODE == 2;
  constexpr bool TRIC = LOWT || UPT;
  // strided batch over blockIdx.y (sA = sB = sC = 0 for a single product)
  A += blockIdx.y * sA;
  B += blockIdx.y * sB;
  C += blockIdx.y * sC;
  // A-side contiguity: no-trans A is m-contiguous; trans A is k-contiguous.
  // B-side as an (n x k) operand: no-trans B is k-contiguous; trans B is n-contiguous.
  constexpr bool AK = TA;
  constexpr bool BKC = !TB;
  using LA = lds_layout<BM, BK, AK>;
  using LB = lds_layout<BN, BK, BKC>;
  // one LDS pool: the K-loop operand tiles, reused by the epilogue to stage
  // the C tile (column chunks of ECH columns, stride BM + 1) so that C is read
  // and written in whole column segments (coalesced 8*BM-byte runs)
  // operand tiles are double-buffered in LDS (one barrier per K stage)
  constexpr int NR = BM == 128 ? 1 : (BM == 64 ? SMG_GEMM_NR64 : SMG_GEMM_NR32);
  constexpr int STAGE = LA::size + LB::size;
  constexpr int OPS = 2 * STAGE;
  constexpr int ECH = (BM * BN + BN <= OPS) ? BN : 32;
  constexpr int POOL = (OPS > (BM + 1) * ECH) ? OPS : (BM + 1) * ECH;
  __shared__ double pool[POOL];

  int bi, bj, tile, split;
  // A triangular operand gives every tile a K range set by its row (op(A))
  // or column (op(B)) block.  The workgroups a CU holds at once are assigned
  // by index, so an order in which that block index varied fastest gave each
  // CU tiles of ONE block: the CUs of the long-K blocks carried ~2x the mean
  // work (N^3 products with a triangular op(A) took 0.88x the full product's
  // time instead of 0.5x).  Such grids run in the linear order (the launch
  // sets px = 0) with that block index varying slowest, longest K first
  // (N = 4096, op(A) upper: 2120 -> 1143 us; op(B) upper 1136 us).
  const bool tri_a_only = !TRIC && (tri & 3) && !(tri & 12);
  const bool tri_b_only = !TRIC && (tri & 12) && !(tri & 3);
  if (px > 0) {
    // XCD-aware placement (full / trapezoidal grids): workgroups b and b + 8
    // share an XCD (round-robin dispatch), so XCD slot x = b % 8 takes one
    // rectangle of a px x (8 / px) partition of the tile grid, column-major
    // inside it; each XCD's L2 then holds 1/px of A's rows and px/8 of B's
    // columns instead of all of both.  Grid: ntp = 8 x the largest rectangle
    // per split; surplus workgroups exit.
    split = blockIdx.x / ntp;
    const int tb = blockIdx.x - split * ntp;
    const int x = tb & 7, l = tb >> 3, py = 8 / px;
    const int tiles_n = ntiles / tiles_m;
    const int rx = x % px, ry = x / px;
    const int r0 = rx * tiles_m / px, r1 = (rx + 1) * tiles_m / px;
    const int c0 = ry * tiles_n / py, c1 = (ry + 1) * tiles_n / py;
    const int rm = r1 - r0;
    if (rm <= 0 || l >= rm * (c1 - c0)) return;
    tile = (r0 + l % rm) + (c0 + l / rm) * tiles_m;
  } else {
    tile = blockIdx.x % ntiles;
    split = blockIdx.x / ntiles;
  }
  // triangle modes: square C -> only the tiles of the triangle are launched
  // (tri_decode); trapezoidal C (m != n, the panel updates of the two-level
  // Cholesky) -> the full grid, tiles wholly outside the triangle exit
  const bool tri_sq = TRIC && m == n && BM == BN;
  if (LOWT && tri_sq) {
    // lower-triangle grids in the order of decreasing K range under the
    // triangular operands (see tri_a_only below): by column (op(B) lower:
    // K in [j0, k)), by column from the right (op(B) upper: K below j0 + BN),
    // by diagonal from the corner (both lower: K in [j0, i0 + BM)), by row
    // from the bottom (op(A) lower alone), else by row from the top
    const int T = tiles_m;
    int r, q;
    if (tri == SMG_TRI_B_LOWER) {
      tri_decode(ntiles - 1 - tile, r, q);
      bj = T - 1 - r;
      bi = bj + q;
    } else if (tri == SMG_TRI_B_UPPER || tri == (SMG_TRI_A_LOWER | SMG_TRI_B_UPPER)) {
      tri_decode(tile, r, q);
      bj = T - 1 - r;
      bi = bj + q;
    } else if (tri == (SMG_TRI_A_LOWER | SMG_TRI_B_LOWER)) {
      tri_decode(tile, r, q);
      bj = q;
      bi = q + (T - 1 - r);
    } else if (tri == SMG_TRI_A_LOWER) {
      tri_decode(ntiles - 1 - tile, bi, bj);
    } else if (tri == 0 && ntiles >= 64) {
      // equal-work tiles (no K cut): XCD x (workgroups b = x mod 8, dispatched
      // round-robin) takes one contiguous run of the grouped tile order, so
      // its L2 holds a few row panels of A and column panels of B at a time
      // (row-major over all XCDs, the last K^{-1} share fetched 530 MB
      // against 151 MB algorithmic, r06 PMC)
      const int b = tile, x = b & 7, per = ntiles >> 3, extra = ntiles & 7;
      tri_decode_grouped(x * per + (x < extra ? x : extra) + (b >> 3), tiles_m, bi, bj);
    } else {
      tri_decode(tile, bi, bj);
    }
  } else if (UPT && tri_sq) {
    tri_decode(tile, bj, bi);
  } else if (tri_a_only) {  // rows slowest, longest K first
    const int r = tile / (ntiles / tiles_m);
    bi = (tri & 1) ? tiles_m - 1 - r : r;
    bj = tile % (ntiles / tiles_m);
  } else if (tri_b_only) {  // columns slowest, longest K first
    const int tn = ntiles / tiles_m, c = tile / tiles_m;
    bi = tile % tiles_m;
    bj = (tri & 8) ? tn - 1 - c : c;
  } else {
    bi = tile % tiles_m;
    bj = tile / tiles_m;
  }
  if (LOWT && !tri_sq && bj * BN > bi * BM + BM - 1) return;
  if (UPT && !tri_sq && bi * BM > bj * BN + BN - 1) return;
  const int i0 = bi * BM, j0 = bj * BN;
  int kbeg = split * kchunk;
  int kend = min(k, kbeg + kchunk);
  if (tri) {
    // triangular operands: only k where both op(A)(i, k) and op(B)(k, j) can
    // be nonzero for some (i, j) of this tile (BK-aligned: the extra
    // elements are stored zeros)
    int lo = 0, hi = k;
    if (tri & 1) hi = min(hi, i0 + BM);  // op(A) lower: zero for k > i
    if (tri & 2) lo = max(lo, i0);       // op(A) upper: zero for k < i
    if (tri & 4) lo = max(lo, j0);       // op(B) lower: zero for k < j
    if (tri & 8) hi = min(hi, j0 + BN);  // op(B) upper: zero for k > j
    lo = lo / BK * BK;
    kbeg = max(kbeg, lo);
    kend = min(kend, hi);
    if (kend < kbeg) kend = kbeg;
  }

  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int NT = 256 * KS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // (kg a compile-time 0 for KS == 1: the fragment reads' LDS offsets fold
  // into immediates; a run-time kg cost the 128 x 128 tile 15 %)
  const int wr = (wave & 3) >> 1, wc = wave & 1, kg = KS == 1 ? 0 : wave >> 2;
  d4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};

  // operand tiles in registers between global memory and LDS: NR sets, so
  // that the load of stage s + NR is in flight while stages s .. s + NR - 1
  // are consumed (NR = 2 for the small tiles, whose grids leave only two or
  // three waves per SIMD to hide the load latency behind)
  constexpr int PA = BM * BK / NT, PB = BN * BK / NT;
  double ra[NR][PA], rb[NR][PB];
  const int nst = (kend - kbeg + BK - 1) / BK;  // K stages of this split
  auto gload = [&](int set, int st) {
    load_tile<BM, BK, AK, NT>(A, lda, m, kend, i0, kbeg + st * BK, ra[set]);
    load_tile<BN, BK, BKC, NT>(B, ldb, n, kend, j0, kbeg + st * BK, rb[set]);
  };
  auto lstore = [&](int set, int buf) {
    store_tile<BM, BK, AK, NT>(pool + buf * STAGE, ra[set]);
    store_tile<BN, BK, BKC, NT>(pool + buf * STAGE + LA::size, rb[set]);
  };
  // every stage load is unconditional (addresses are clamped in range and
  // stages past the end are masked to zero): a conditional load would make
  // the waitcnt pass assume the worst on the loop back-edge and wait for ALL
  // outstanding loads at each LDS store, i.e. no prefetch at all
#pragma unroll
  for (int j = 0; j < NR; ++j) gload(j, j);
  // epilogue operand in flight during the K loop (small tiles only: the
  // 128 x 128 tile would double its register count); coalesced mapping
  // e = tid + 256 q -> (i = e % BM, j = e / BM), the same as the store
  constexpr int EPT = BM * BN / NT;
  constexpr bool PREFETCH_C = EPT <= 16;
  // bz: tiles from row bz (bz > 0) or column -bz (bz < 0) on take beta = 0
  // (the first contribution to a region of an accumulated product: C is not read)
  const bool use_c = !slab && beta != 0.0 && !(bz > 0 && i0 >= bz) && !(bz < 0 && j0 >= -bz);
  double cpre[PREFETCH_C ? EPT : 1];
  if (PREFETCH_C) {
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = threadIdx.x + NT * q;
      const int i = i0 + e % BM, j = j0 + e / BM;
      cpre[q] = (use_c && i < m && j < n) ? C[i + (size_t)j * ldc] : 0.0;
    }
  }
  const int fr = lane & 15, fk = lane >> 4;
  static_assert(BK / 4 % KS == 0, "K stage split");
  auto mma_stage = [&](const double* Ab, const double* Bb) {
#pragma unroll
    for (int kq = 0; kq < BK / 4 / KS; ++kq) {
      const int ks = kg * (BK / 4 / KS) + kq;
      double af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[a] = Ab[LA::at(wr * (BM / 2) + a * 16 + fr, ks * 4 + fk)];
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bf[b] = Bb[LB::at(wc * (BN / 2) + b * 16 + fr, ks * 4 + fk)];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
  };
  // stage s computes from LDS buffer s & 1 while stage s + 1 is stored into
  // the other buffer and stage s + 1 + NR is issued into the freed registers
  // (one barrier per stage); the loop is unrolled by two so that every
  // register-set index is a compile-time constant
  // (an odd stage count runs one all-zero stage: the loop body has no
  // conditional memory operations)
  lstore(0, 0);
  gload(0, NR);
  __syncthreads();
  // stage st: MMA from LDS buffer st & 1, store stage st + 1 (register set
  // (st + 1) % NR) into the other buffer, refill that set with stage
  // st + 1 + NR.  Unrolled by U = lcm(2, NR) so every set / buffer index is a
  // compile-time constant; the main loop has no conditional memory operation
  // (the tail's guards only cost precision of its own waits).
  constexpr int U = NR % 2 == 0 ? NR : 2 * NR;
  auto body = [&](int st, auto uc) {
    constexpr int u = decltype(uc)::value;
    mma_stage(pool + (u & 1) * STAGE, pool + (u & 1) * STAGE + LA::size);
    lstore((u + 1) % NR, (u & 1) ^ 1);
    gload((u + 1) % NR, st + 1 + NR);
    __syncthreads();
  };
  int s0 = 0;
  for (; s0 + U <= nst; s0 += U)
    smg_static_for<U>([&](auto uc) { body(s0 + decltype(uc)::value, uc); });
  smg_static_for<U - 1>([&](auto uc) {
    if (s0 + decltype(uc)::value < nst) body(s0 + decltype(uc)::value, uc);
  });

  // epilogue: D layout of v_mfma_f64_16x16x4_f64: reg r of lane l holds
  // row (l>>4) + 4r, col l&15 of the 16x16 tile.  Accumulators go to LDS
  // (column-major, stride BM + 1), then every thread stores whole column runs.
  __syncthreads();  // operand tiles no longer needed
#pragma unroll
  for (int c0 = 0; c0 < BN; c0 += ECH) {
    // k-group 0 stores its accumulators, the other groups add theirs in turn
#pragma unroll
    for (int g = 0; g < KS; ++g) {
      if (kg == g) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            const int jl = wc * (BN / 2) + b * 16 + (lane & 15) - c0;
            if (jl < 0 || jl >= ECH) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              double* d = &pool[jl * (BM + 1) + wr * (BM / 2) + a * 16 + (lane >> 4) + 4 * r];
              *d = g == 0 ? acc[a][b][r] : *d + acc[a][b][r];
            }
          }
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < BM * ECH / NT; ++q) {
      const int e = threadIdx.x + NT * q;
      const int il = e % BM, jl = e / BM;
      const int i = i0 + il, j = j0 + c0 + jl;
      if (i >= m || j >= n) continue;
      if (LOWT && i < j) {
        if (MODE == 3 && C2) C2[i + (size_t)j * ldc2] = 0.0;  // (Phi's zero upper inside the diagonal tiles)
        continue;
      }
      if (UPT && i > j) continue;
      const double v = pool[jl * (BM + 1) + il];
      if (slab) {
        slab[(size_t)split * m * n + (size_t)j * m + i] = v;
      } else {
        double out;
        if (!use_c) {
          out = alpha * v;
        } else {
          double cv;
          if (PREFETCH_C) cv = cpre[(c0 / ECH) * (BM * ECH / NT) + q];
          else cv = C[i + (size_t)j * ldc];
          out = alpha * v + beta * cv;
        }
        C[i + (size_t)j * ldc] = out;
        if (MODE == 3 && i > j) C[j + (size_t)i * ldc] = out;
        if ((MODE == 4 || (MODE == 3 && C2)) && i >= j) C2[i + (size_t)j * ldc2] = i == j ? 0.5 * out : out;
      }
    }
    if (c0 + ECH < BN) __syncthreads();
  }
}

__global__ void k_splitk_reduce(int m, int n, int splits, const double* __restrict__ slab,
                                double alpha, double beta, double* __restrict__ C,
                                int ldc, int lower, int bz) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)m * n) return;
  const int i = (int)(idx % m), j = (int)(idx / m);
  if (lower == 1 && i < j) return;
  if (lower == 2 && i > j) return;
  double s = 0.0;
  for (int t = 0; t < splits; ++t) s += slab[(size_t)t * m * n + idx];
  double* c = C + i + (size_t)j * ldc;
  if ((bz > 0 && i >= bz) || (bz < 0 && j >= -bz)) beta = 0.0;  // (k_gemm's bz)
  *c = (beta == 0.0) ? alpha * s : alpha * s + beta * *c;
}

// the same reduction for an even m: a lane takes two rows of one column
// (16-byte slab loads, every split's load issued before the sum), a 2-D
// grid-stride walk instead of a 64-bit division per element, a bounded grid
// (the per-element form spent most of its time on index arithmetic: 44 us for
// four 512 x 2560 slabs)
__global__ __launch_bounds__(256) void k_splitk_reduce2(int m, int n, int splits, const double* __restrict__ slab,
                                                        double alpha, double beta, double* __restrict__ C, int ldc,
                                                        int lower, int bz) {
  const long long tot = (long long)m * n;
  for (smg_mn w(m >> 1, n); w.ok(); w.next()) {
    const int i = 2 * w.i, j = w.j;
    if (lower == 1 && i + 1 < j) continue;
    if (lower == 2 && i > j) continue;
    const long long e = (long long)j * m + i;
    d2v s = {0.0, 0.0};
    int t = 0;
    for (; t + 4 <= splits; t += 4) {
      const d2v a0 = *reinterpret_cast<const d2v*>(slab + (size_t)t * tot + e);
      const d2v a1 = *reinterpret_cast<const d2v*>(slab + (size_t)(t + 1) * tot + e);
      const d2v a2 = *reinterpret_cast<const d2v*>(slab + (size_t)(t + 2) * tot + e);
      const d2v a3 = *reinterpret_cast<const d2v*>(slab + (size_t)(t + 3) * tot + e);
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; t < splits; ++t) s += *reinterpret_cast<const d2v*>(slab + (size_t)t * tot + e);
    double* c = C + i + (size_t)j * ldc;
    const bool w0 = !(lower == 1 && i < j), w1 = !(lower == 2 && i + 1 > j);
    // (k_gemm's bz; an even row boundary keeps both rows of the pair on one side)
    const double b = ((bz > 0 && i >= bz) || (bz < 0 && j >= -bz)) ? 0.0 : beta;
    if (w0) c[0] = (b == 0.0) ? alpha * s[0] : alpha * s[0] + b * c[0];
    if (w1) c[1] = (b == 0.0) ? alpha * s[1] : alpha * s[1] + b * c[1];
  }
}

// the second output of MODE 4 (launch reads it from here: one product at a
// time per host thread issues a MODE-4 GEMM)
thread_local double* t_c2 = nullptr;
thread_local int t_ldc2 = 0;
// the beta-zero boundary of the next product (k_gemm's bz; smg_gemm_bz_impl)
thread_local int t_bz = 0;

template <int BM, int BN, int BK, bool TA, bool TB, int MODE, int KS = 1>
int launch(smg_ctx* ctx, int m, int n, int k, double alpha, const double* A,
           int lda, const double* B, int ldb, double beta, double* C, int ldc, int batch = 1,
           long long sA = 0, long long sB = 0, long long sC = 0, int tri = 0) {
  constexpr bool TRIC = MODE == 1 || MODE == 2 || MODE == 3;
  const int tm = smg_ceil_div(m, BM), tn = smg_ceil_div(n, BN);
  const int ntiles = (TRIC && m == n && BM == BN) ? tm * (tm + 1) / 2 : tm * tn;
  // split K when the tile grid cannot fill the 256 CUs and K is long
  int splits = 1;
  const int target = 512;
  constexpr int KMIN = 64;  // shortest K chunk of a split
  // (a grid that already covers every CU once keeps K whole while K is short:
  // 512^3 with 32 x 32 tiles, 256 tiles: 12.3 us unsplit vs 15.9 us split
  // in two plus the reduction)
  const bool covers = ntiles >= 256 && k <= 1024;
  // (triangular operands: every tile has its own K range, no split)
  // (MODE 3 / 4 products -- the symbolic step's, with triangular operands --
  // never split)
  if (!tri && MODE != 3 && MODE != 4 && batch == 1 && ntiles < target && !covers &&
      k >= 2 * KMIN) {
    splits = smg_ceil_div(target, ntiles);
    const int maxs = k / KMIN;
    if (splits > maxs) splits = maxs;
    if (splits > 64) splits = 64;
    if (splits < 1) splits = 1;
  }
  int kchunk = smg_ceil_div(smg_ceil_div(k, splits), BK) * BK;
  splits = smg_ceil_div(k, kchunk);
  double* slab = nullptr;
  if (splits > 1) {
    // the side and zeroing streams have their own slabs so concurrent split-K
    // GEMMs never share one
    const int slot = ctx->stream == ctx->side                                ? SMG_WS_GEMM_SIDE
                     : (ctx->zero_stream && ctx->stream == ctx->zero_stream) ? SMG_WS_GEMM_ZERO
                                                                             : SMG_WS_GEMM;
    slab = smg_ws(ctx, slot, (size_t)splits * m * n);
    if (!slab) return SMG_ERR_OOM;
  }
  // XCD partition px x (8 / px) of a full tile grid minimising the per-XCD
  // operand footprint (rows of A + columns of B, in tiles); triangle grids
  // (tri_decode order) and grids too small to split keep the linear order
  // (a triangular operand alone: the linear, longest-K-first order of the
  // kernel's tile decode instead)
  const bool tri_one = !TRIC && tri && (!(tri & 3) || !(tri & 12));
  int px = 0, ntp = ntiles;
  if (!(TRIC && m == n && BM == BN) && ntiles >= 64 && !tri_one) {
    long long best = -1;
    for (int p = 1; p <= 8; p *= 2) {
      const int q = 8 / p;
      if (p > tm || q > tn) continue;
      const long long rr = smg_ceil_div(tm, p), cc = smg_ceil_div(tn, q);
      const long long foot = rr * BM + cc * BN;
      if (best < 0 || foot < best) {
        best = foot;
        px = p;
        ntp = 8 * (int)(rr * cc);
      }
    }
  }
  hipLaunchKernelGGL((k_gemm<BM, BN, BK, TA, TB, MODE, KS>), dim3(ntp * splits, batch), dim3(256 * KS), 0,
                     ctx->stream, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tm,
                     ntiles, kchunk, slab, sA, sB, sC, px, ntp, tri, MODE >= 3 ? t_c2 : nullptr,
                     MODE >= 3 ? t_ldc2 : 0, t_bz);
  if (splits > 1) {
    const long long tot = (long long)m * n;
    if ((m & 1) == 0) {
      const long long pairs = tot / 2;
      const int nb = (int)(pairs / 256 < 2048 ? (pairs + 255) / 256 : 2048);
      hipLaunchKernelGGL(k_splitk_reduce2, dim3(nb), dim3(256), 0, ctx->stream, m, n, splits, slab, alpha, beta,
                         C, ldc, MODE, t_bz);
    } else {
      hipLaunchKernelGGL(k_splitk_reduce, dim3(smg_ceil_div(tot, 256)), dim3(256), 0,
                         ctx->stream, m, n, splits, slab, alpha, beta, C, ldc, MODE, t_bz);
    }
  }
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

// Do two column-major blocks share an element?  Blocks with the same leading
// dimension are treated as rectangles of one matrix (the sub-blocks Murray's
// reverse works on: La[k:, j:k] vs La[j:k, 0:k] are disjoint although their
// address ranges interleave); otherwise the address ranges are compared.
inline bool overlaps(const double* X, int ldx, int rows, int cols, const double* C, int ldc, int m,
                     int n) {
  if (rows <= 0 || cols <= 0 || m <= 0 || n <= 0) return false;
  const double* x1 = X + (size_t)(cols - 1) * ldx + rows;
  const double* c1 = C + (size_t)(n - 1) * ldc + m;
  if (!(X < c1 && C < x1)) return false;
  if (ldx != ldc) return true;
  const double* base = X < C ? X : C;
  const long long ox = X - base, oc = C - base, ld = ldx;
  const long long rx = ox % ld, cx = ox / ld, rc = oc % ld, cc = oc / ld;
  return rx < rc + m && rc < rx + rows && cx < cc + n && cc < cx + cols;
}

// K stage of the 64 x 64 tile: 16 keeps two stages of registers and two LDS
// buffers within 32 KB per workgroup (four or more workgroups per CU)
constexpr int BK64 = 16;

template <bool TA, bool TB, int MODE>
int dispatch_tile(smg_ctx* ctx, int m, int n, int k, double alpha, const double* A,
                  int lda, const double* B, int ldb, double beta, double* C, int ldc, int tri) {
  constexpr bool FULLC = MODE == 0 || MODE == 4;  // every tile of C computed
  // In-place products (C aliases an operand: the blocked TRSMs C = C Dinv,
  // L21 = A21 Dinv^T, X_p = W_p B_p) are race-free only when every workgroup
  // owns whole rows (C aliases A) or whole columns (C aliases B) of C.
  const bool alias_a = overlaps(A, lda, TA ? k : m, TA ? m : k, C, ldc, m, n);
  const bool alias_b = overlaps(B, ldb, TB ? n : k, TB ? k : n, C, ldc, m, n);
  if (alias_a || alias_b) {
    if (MODE == 3 || MODE == 4 || t_bz) return SMG_ERR_ARG;  // (the symbolic step's products never alias)
    if (MODE == 0 && alias_a && !alias_b && n <= 64)
      return launch<32, 64, 32, TA, TB, 0>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, 0, 0, tri);
    if (MODE == 0 && alias_b && !alias_a && m <= 64)
      return launch<64, 32, 32, TA, TB, 0>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, 0, 0, tri);
    // general aliasing: out of place through a workspace, then C = T (+ beta C)
    double* T = smg_ws(ctx, SMG_WS_ALIAS, (size_t)m * n);
    if (!T) return SMG_ERR_OOM;
    int rc = dispatch_tile<TA, TB, MODE>(ctx, m, n, k, alpha, A, lda, B, ldb, 0.0, T, m, tri);
    if (rc) return rc;
    if (beta == 0.0) return smg_copy_impl(ctx, m, n, T, m, C, ldc, 1.0, 0);
    if (beta != 1.0) {
      rc = smg_scale_impl(ctx, m, n, beta, C, ldc, MODE);
      if (rc) return rc;
    }
    return smg_copy_impl(ctx, m, n, T, m, C, ldc, 1.0, 1);
  }
  // tile size by how many CUs the output grid can occupy (256 CUs): large
  // outputs take 128x128 tiles (operand reuse), mid-size 64x64, and the
  // CU-starved shapes of the blocked Cholesky (one 64-wide block column or
  // row) 32x32, so the grid spreads over 4x more CUs
  const long long big_tiles = (long long)smg_ceil_div(m, 128) * smg_ceil_div(n, 128);
  const long long t64 = smg_ceil_div(m, 64);
  const long long mid_tiles =
      (!FULLC && m == n) ? t64 * (t64 + 1) / 2 : t64 * smg_ceil_div(n, 64);
  // (triangle modes keep 64 x 64 tiles: half the 128-tile grid would sit on
  // the diagonal, and the split-K those few tiles need costs a reduction; at
  // N = K = 4096 the 528-tile 128 triangle -- 2.06 waves over the CUs -- ran
  // 1692 vs 1416 us for the 64 grid)
  // (a triangular operand gives the tiles K ranges from 128 to k: with one
  // 128 tile per CU the longest sets the time -- the 2048^3 products of the
  // inverse doubling ran at 27 TF/s -- so those need 4 per CU to balance,
  // else the 64 x 64 grid's longest-K-first order takes them)
  if (FULLC && big_tiles >= (tri ? SMG_GEMM_TRI128_MIN : 256) && k > 128)
    return launch<128, 128, 16, TA, TB, MODE>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, 0, 0, tri);
  // long-K transposed-A products with a small output (the Murray reverse's
  // [R_adj | D_adj] -= C_adj^T [B | C]: 512 x K x m, m >= 1536): 128 x 64
  // tiles split over K (tools/ubench_gemm: (512,2048,2048) 87 vs 100 us,
  // (512,1024,3072) 68 vs 81 us with 32 x 32)
  if (MODE == 0 && TA && !TB && k >= 1536 && mid_tiles < 512)
    return launch<128, 64, 16, TA, TB, MODE>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, 0, 0, tri);
  // 64 x 64 tiles from 256 tiles on (one per CU), with 8 waves (KS = 2: the
  // two wave groups split every K stage) up to ~6 tiles per CU; 32 x 32
  // below that (4x the workgroups), and for the tall NN products with
  // n <= 512 (C_adj D^{-1}, B_adj -= C_adj R at small J), where the
  // 4-wave 32 x 32 grid measured fastest.  tools/ubench_gemm at N = 4096
  // (us, 32x32 / 64x64 / 64x64 KS=2):
  //   (3584,512,512) NT lower 57.6 / 54.6 / 51.4   (512,3584,512) NN 49.6 / 51.8 / 47.3
  //   (2048,1536,512) NN 80.5 (64x64) / 70.6       (3072,512,512) NN 45.1 / 52.5 / 48.4
  //   (512,512,512) 11.5 (32x32) / 10.2 (32x32 KS=2)
  // (and a 64 x 64 grid below 256 tiles, split over K or not, loses to 32 x 32:
  // (3584,256,256) 18.6 vs 28 us)
  if (mid_tiles >= 512) {
    if (mid_tiles <= SMG_GEMM_KS2_MAX)
      return launch<64, 64, BK64, TA, TB, MODE, 2>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, 0, 0, tri);
    return launch<64, 64, BK64, TA, TB, MODE>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, 0, 0, tri);
  }
  const bool tall_nn = MODE == 0 && !TA && !TB && n <= 512;
  if (mid_tiles >= 256 && !tall_nn)
    return launch<64, 64, BK64, TA, TB, MODE, 2>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, 0, 0, tri);
  const long long t32 = smg_ceil_div(m, 32);
  const long long small_tiles = (!FULLC && m == n) ? t32 * (t32 + 1) / 2 : t32 * smg_ceil_div(n, 32);
  if (small_tiles <= 256)
    return launch<32, 32, 32, TA, TB, MODE, 2>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, 0, 0, tri);
  return launch<32, 32, 32, TA, TB, MODE>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, 1, 0, 0, 0, tri);
}

}  // namespace

// batch x (C_i = alpha op(A_i) op(B_i) + beta C_i), operand i at base + i * stride
// (doubles); full C only, no split-K, operands must not alias
int smg_gemm_batched_impl(smg_ctx* ctx, int ta, int tb, int m, int n, int k, double alpha,
                          const double* A, int lda, long long sA, const double* B, int ldb,
                          long long sB, double beta, double* C, int ldc, long long sC, int batch) {
  if (m <= 0 || n <= 0 || batch <= 0) return SMG_OK;
  if (k <= 0 || alpha == 0.0) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GEMM);
  if (ctx->prof_on) ctx->prof_flops[SMG_FAM_GEMM] += 2.0 * m * n * k * batch;
  const bool big = (long long)smg_ceil_div(m, 64) * smg_ceil_div(n, 64) * batch >= 192;
#define SMG_BATCHED(TA_, TB_)                                                                    \
  return big ? launch<64, 64, BK64, TA_, TB_, 0>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, \
                                               batch, sA, sB, sC)                                 \
             : launch<32, 32, 32, TA_, TB_, 0>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, \
                                               batch, sA, sB, sC);
  if (!ta && !tb) SMG_BATCHED(false, false)
  if (!ta && tb) SMG_BATCHED(false, true)
  if (ta && !tb) SMG_BATCHED(true, false)
  SMG_BATCHED(true, true)
#undef SMG_BATCHED
}

int smg_gemm_impl(smg_ctx* ctx, int ta, int tb, int uplo, int m, int n, int k,
                  double alpha, const double* A, int lda, const double* B, int ldb,
                  double beta, double* C, int ldc, int tri) {
  if (m <= 0 || n <= 0) return SMG_OK;
  if (k <= 0 || alpha == 0.0) {
    if (beta == 1.0) return SMG_OK;
    return smg_scale_impl(ctx, m, n, beta, C, ldc, uplo);
  }
  smg_prof_scope prof(ctx, SMG_FAM_GEMM);
  if (ctx->prof_on) {
    // the K cuts of triangular operands execute about half (one) or a third
    // (two, as in V V^T with a triangle output) of the dense count
    const double cut = (tri & 3) && (tri & 12) ? 1.0 / 3.0 : (tri ? 0.5 : 1.0);
    ctx->prof_flops[SMG_FAM_GEMM] +=
        cut * (uplo ? 2.0 * k * ((double)m * n - (double)n * (n - 1) / 2) : 2.0 * m * n * k);
  }
  if (uplo == 1) {
    if (!ta && tb) return dispatch_tile<false, true, 1>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
    if (ta && !tb) return dispatch_tile<true, false, 1>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
    if (!ta && !tb) return dispatch_tile<false, false, 1>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
    return dispatch_tile<true, true, 1>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  }
  if (uplo == 3) {  // lower half computed, stored mirrored (symmetric C)
    if (ta && !tb) return dispatch_tile<true, false, 3>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
    if (!ta && !tb) return dispatch_tile<false, false, 3>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
    if (!ta && tb) return dispatch_tile<false, true, 3>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
    return dispatch_tile<true, true, 3>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  }
  if (uplo == 2) {
    if (!ta && tb) return dispatch_tile<false, true, 2>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
    if (ta && !tb) return dispatch_tile<true, false, 2>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
    if (!ta && !tb) return dispatch_tile<false, false, 2>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
    return dispatch_tile<true, true, 2>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  }
  if (!ta && !tb) return dispatch_tile<false, false, 0>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  if (!ta && tb) return dispatch_tile<false, true, 0>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  if (ta && !tb) return dispatch_tile<true, false, 0>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  return dispatch_tile<true, true, 0>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
}

// smg_gemm_impl with beta taken as 0 for C's rows from bz on (bz > 0) or its
// columns from -bz on (bz < 0): the first contribution to that region of an
// accumulated product, which then needs no zeroing beforehand.  |bz| must be a
// multiple of 128 (every tile lies on one side of it).
int smg_gemm_bz_impl(smg_ctx* ctx, int ta, int tb, int uplo, int m, int n, int k, double alpha, const double* A,
                     int lda, const double* B, int ldb, double beta, double* C, int ldc, int tri, int bz) {
  if (bz % 128) return SMG_ERR_ARG;
  t_bz = bz;
  const int rc = smg_gemm_impl(ctx, ta, tb, uplo, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  t_bz = 0;
  return rc;
}

// C = alpha op(A) op(B) + beta C (full) and C2 = tril(C) with halved diagonal
int smg_gemm_dual_impl(smg_ctx* ctx, int ta, int tb, int m, int n, int k, double alpha, const double* A, int lda,
                       const double* B, int ldb, double beta, double* C, int ldc, double* C2, int ldc2, int tri) {
  if (m <= 0 || n <= 0) return SMG_OK;
  if (k <= 0 || alpha == 0.0 || !C2) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GEMM);
  if (ctx->prof_on) ctx->prof_flops[SMG_FAM_GEMM] += 2.0 * m * n * k;
  t_c2 = C2;
  t_ldc2 = ldc2;
  int rc;
  if (!ta && !tb) rc = dispatch_tile<false, false, 4>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  else if (ta && !tb) rc = dispatch_tile<true, false, 4>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  else if (!ta && tb) rc = dispatch_tile<false, true, 4>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  else rc = dispatch_tile<true, true, 4>(ctx, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  t_c2 = nullptr;
  return rc;
}

// C = alpha op(A) op(B) + beta C, symmetric: its lower triangle computed and
// stored mirrored (uplo 3), and P = Phi(C) (strict lower, halved diagonal) as
// a second output.  P's strict upper is written (zeros) only inside the
// diagonal tiles: a reader must cut K to P's lower triangle
// (SMG_TRI_B_LOWER / TRI_B_UPPER on P^T), as the Cholesky tangent's do.
int smg_gemm_sym_phi_impl(smg_ctx* ctx, int ta, int tb, int n, int k, double alpha, const double* A, int lda,
                          const double* B, int ldb, double beta, double* C, int ldc, double* P, int ldp, int tri) {
  if (n <= 0) return SMG_OK;
  if (k <= 0 || alpha == 0.0 || !P) return SMG_ERR_ARG;
  smg_prof_scope prof(ctx, SMG_FAM_GEMM);
  if (ctx->prof_on) {
    const double cut = (tri & 3) && (tri & 12) ? 1.0 / 3.0 : (tri ? 0.5 : 1.0);
    ctx->prof_flops[SMG_FAM_GEMM] += cut * 2.0 * k * ((double)n * n - (double)n * (n - 1) / 2);
  }
  t_c2 = P;
  t_ldc2 = ldp;
  int rc;
  if (!ta && !tb) rc = dispatch_tile<false, false, 3>(ctx, n, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  else if (ta && !tb) rc = dispatch_tile<true, false, 3>(ctx, n, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  else if (!ta && tb) rc = dispatch_tile<false, true, 3>(ctx, n, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  else rc = dispatch_tile<true, true, 3>(ctx, n, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
  t_c2 = nullptr;
  return rc;
}

extern "C" int smg_gemm_tri(smg_ctx* ctx, int ta, int tb, int uplo, int tri, int m, int n, int k,
                            double alpha, const double* A, int lda, const double* B, int ldb, double beta,
                            double* C, int ldc) {
  if (!ctx || m < 0 || n < 0 || k < 0 || tri < 0 || tri > 15) return SMG_ERR_ARG;
  if ((m > 0 && n > 0) && (!C || ldc < m)) return SMG_ERR_ARG;
  if (k > 0 && m > 0 && n > 0 && alpha != 0.0) {
    if (!A || !B) return SMG_ERR_ARG;
    if (lda < (ta ? k : m) || ldb < (tb ? n : k)) return SMG_ERR_ARG;
  }
  return smg_gemm_impl(ctx, ta, tb, uplo, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, tri);
}

extern "C" int smg_gemm(smg_ctx* ctx, int ta, int tb, int uplo, int m, int n, int k,
                        double alpha, const double* A, int lda, const double* B,
                        int ldb, double beta, double* C, int ldc) {
  if (!ctx || m < 0 || n < 0 || k < 0) return SMG_ERR_ARG;
  if ((m > 0 && n > 0) && (!C || ldc < m)) return SMG_ERR_ARG;
  if (k > 0 && m > 0 && n > 0 && alpha != 0.0) {
    if (!A || !B) return SMG_ERR_ARG;
    if (lda < (ta ? k : m) || ldb < (tb ? n : k)) return SMG_ERR_ARG;
  }
  return smg_gemm_impl(ctx, ta, tb, uplo, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc);
}

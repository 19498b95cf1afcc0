// Fused spatial graph convolution, bf16 path (STGCN_F_BF16) — gfx950 only.
//
// k_sp_fwd_bf16<V, K>: the whole SpatialConv of the block in one kernel,
//   Z[n, co, t, v] = sum_k sum_ci W_k[co, ci] * G_k[n, ci, t, v] + biasZ[co, v],
//   G_k[n, ci, t, v] = sum_w A_k[v, w] * f(BN1(x))[n, ci, t, w]
// (st_graphconv.py:98 BN1, :139-152 SpatialConv in the form (1) of capi.hip;
// f = ReLU for the residual block, :72-74). The joint contraction runs on the
// matrix cores with A pinned in LDS, so the K*C_in-channel G is never written to
// and read back from HBM in fp32 (the unfused path: k_gather_mfma writes G,
// k_conv_bf16<1,...> reads it):
//   per workgroup: clip n, FT = 256/V frames, 64 output channels (row tile);
//   per chunk of 16 input channels:
//     X  = bf16(f(BN1(x)))  [row = t*16 + ch][w]            (staged from HBM)
//     G  = X * (Ah + Am)^T  on v_mfma_f32_32x32x16_bf16, A as two exact bf16
//          planes (A = Ah + Am to 2^-16): rows (t, ch) x cols (k, v), k-dim w
//     G  -> bf16 image [position t*V + v][k*16 + ch] (16-byte octet slots,
//          2K+1 slots per position: odd, ds_read_b128 conflict-free)
//     Z += W'(chunk) * G    on v_mfma_f32_32x32x16_bf16 (the W' GEMM; packed
//          bf16 weights [chunk][k][octet][64 rows][8] by LDS-DMA)
//   epilogue: conv_tile_epilogue (bias table, BN2 statistics of the residual
//   block), Z in fp32.
// Numerics: the same roundings as the reference run with bf16 conv operands
// (BN1(x) and W rounded to bf16, fp32 accumulation) plus G rounded to bf16 as
// the W' GEMM operand (as in the unfused bf16 path); A enters exactly to 2^-16.
// Optionally (Gk != null, row-tile 0 only) the bf16 G image is also written to
// HBM for the backward weight gradient dW' = dZ G^T, in the layout
//   Gk[n][k*C_in + ci][mtile][256 positions]   (positions >= NCOLS are zero)
// i.e. half the bytes of the fp32 G and already the operand precision the
// bf16 weight gradient uses (k_wgrad_gemm_bf16 rounds G to bf16 at read).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "internal.h"

namespace stgcn {

typedef __bf16 bf16x8f __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2f __attribute__((ext_vector_type(2)));
typedef int int4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ floatx16 mfma_bf(bf16x8f a, bf16x8f b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ unsigned pkbf(float a, float b) {
  const bf16x2f v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}

template <int V, int K>
struct SpFwdGeo {
  static constexpr int FT = kTileCols / V;
  static constexpr int NCOLS = FT * V;
  static constexpr int CK = 16;                    // input channels per chunk
  static constexpr int XROWS = CK * FT;            // gather rows (t, ch)
  static constexpr int RT = (XROWS + 31) / 32;     // gather row tiles
  static constexpr int KW = (V + 15) & ~15;        // gather reduction (joints w), padded
  static constexpr int KS = KW / 16;               // gather k-steps
  static constexpr int XP = KW + 8;                // X / A image pitch (bf16): conflict-free b128
  static constexpr int NGC = K * V;                // gather columns (k, v)
  static constexpr int GC = (NGC + 31) / 32;       // gather column tiles
  static constexpr int GT = RT * GC;               // gather tiles
  static constexpr int SLOTS = 2 * K + 1;          // G image 16-byte slots per position
  static constexpr int X_BYTES = RT * 32 * XP * 2;
  static constexpr int A_BYTES = GC * 32 * XP * 2;  // one plane
  static constexpr int G_BYTES = NCOLS * SLOTS * 16;
  static constexpr int W_BYTES = K * 2 * 1024;     // packed W' chunk
  static constexpr int NIT = CK * NCOLS;           // x staging items (ch, pos)
  static constexpr int IPT = (NIT + 255) / 256;
  // layout: [A h][A m][X][G][W0][W1][BN tables 2 x 3 x 16 floats]
  static constexpr int A_IMG = (2 * A_BYTES + 1023) & ~1023;  // both planes, whole KiB
  static constexpr int OFF_AH = 0, OFF_AM = A_BYTES, OFF_X = A_IMG;
  static constexpr int OFF_G = OFF_X + X_BYTES, OFF_W = OFF_G + G_BYTES;
  static constexpr int OFF_BN = OFF_W + 2 * W_BYTES;
  static constexpr int LDS = OFF_BN + 2 * 6 * 16 * 4;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(LDS >= 2048 + 64 * V * 4, "epilogue scratch fits");
  static_assert(IPT <= 16, "staging registers");
};

struct SpFwdParams {
  const float *x, *mean, *invstd, *g, *b, *A;
  // ABI 8 (STGCN_PLAN_X_FROM_U; pmean non-null): x holds the previous block's U
  // and the input is ReLU(BN2_prev(U)), formed on staging as k_bn_relu_fwd forms
  // its y (the previous block then writes only y's statistics)
  const float *pmean, *pinvstd, *pg, *pb;
  const __bf16 *aimg;  // the LDS image of the A planes (k_pack_sp_a), DMA'd per workgroup
  const __bf16 *wpk;  // [rt][chunk][k][octet][64][8]
  __bf16 *Gk;         // optional kept G (bf16 tile layout), or null
  int C, T, relu, nchunks;
  ConvGemmParams ep;  // epilogue: out = Z, bias_rv, stats, R, V, M, T_dst, tiles
};

#define SPF_ST16(k)                                                                        \
  "+v"(st[k + 0]), "+v"(st[k + 1]), "+v"(st[k + 2]), "+v"(st[k + 3]), "+v"(st[k + 4]),   \
      "+v"(st[k + 5]), "+v"(st[k + 6]), "+v"(st[k + 7])
__device__ __forceinline__ void spf_wait_all(float (&st)[16]) {
  asm volatile("s_waitcnt vmcnt(0)" : SPF_ST16(0), SPF_ST16(8)::"memory");
}
#undef SPF_ST16

template <int V, int K>
__global__ __launch_bounds__(256, 2) void k_sp_fwd_bf16(SpFwdParams P) {
  using G = SpFwdGeo<V, K>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const ConvGemmParams &p = P.ep;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = bid % p.n_rtiles;
  bid /= p.n_rtiles;
  const int mt = bid % p.n_mtiles;
  const int n = bid / p.n_mtiles;
  const int r0 = rt * kTileRows, m0 = mt * G::FT;
  const int TV = P.T * V;
  const int nch = P.nchunks;

  // ---- prologue: A planes (h, m) by 16-byte LDS-DMA of the prebuilt image
  // (k_pack_sp_a), zeroed X pads; landed by the vmcnt(0) before the first barrier
  {
    const __amdgpu_buffer_rsrc_t ra =
        make_rsrc(reinterpret_cast<const float *>(P.aimg), G::A_IMG / 4);
    for (int i = wave; i < G::A_IMG / 1024; i += 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, smem + i * 256, 16,
                                               (unsigned)(i * 1024 + lane * 16), 0, 0, 0);
    unsigned *xz = reinterpret_cast<unsigned *>(lds + G::OFF_X);
    for (int e = tid; e < G::X_BYTES / 4; e += 256) xz[e] = 0u;
  }
  // ---- x staging: items (ch, pos), consecutive threads = consecutive positions
  const uint64_t xsrc = reinterpret_cast<uint64_t>(P.x + (int64_t)n * P.C * TV);
  int loff[G::IPT];     // X image element offset (-1: no item)
  unsigned goff[G::IPT];  // byte offset within the chunk's first channel (kOOB: zero)
  int ich[G::IPT];
#pragma unroll
  for (int k = 0; k < G::IPT; ++k) {
    const int e = k * 256 + tid;
    const int ch = e / G::NCOLS, pos = e - ch * G::NCOLS;
    const int t = pos / V, w = pos - t * V;
    const bool live = e < G::NIT;
    loff[k] = live ? (t * 16 + ch) * G::XP + w : -1;
    ich[k] = live ? ch : 0;
    goff[k] = (live && m0 * V + pos < TV) ? (unsigned)((ch * TV + m0 * V + pos) * 4) : kOOB;
  }
  float st[16];
  auto load_x = [&](int chunk) {
    const int64_t rem = (int64_t)(P.C - chunk * G::CK) * TV * 4;
    const uint64_t src = xsrc + (uint64_t)chunk * G::CK * TV * 4;
    const int4f rs = {(int)(uint32_t)src, (int)((src >> 32) & 0xffff),
                      (int)(rem > 0x7fffffff ? 0x7fffffff : (rem > 0 ? rem : 0)), 0x00020000};
    asm volatile("s_nop 4" ::: "memory");
#pragma unroll
    for (int k = 0; k < G::IPT; ++k)
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen"
                   : "=v"(st[k])
                   : "v"(goff[k]), "s"(rs)
                   : "memory");
  };
  float *bnt = reinterpret_cast<float *>(lds + G::OFF_BN);  // [2][6][16]: mean, a, beta; prev
  auto bn_table = [&](int chunk, int slot) {
    if (tid < 16) {
      const int c = chunk * G::CK + tid;
      float mu = 0.f, a = 0.f, be = 0.f, pmu = 0.f, pa = 0.f, pbe = 0.f;
      if (c < P.C) {
        mu = P.mean[c];
        a = P.invstd[c] * P.g[c];
        be = P.b[c];
        if (P.pmean) {
          pmu = P.pmean[c];
          pa = P.pinvstd[c] * P.pg[c];
          pbe = P.pb[c];
        }
      }
      float *tb = bnt + slot * 96;
      tb[tid] = mu;
      tb[16 + tid] = a;
      tb[32 + tid] = be;
      tb[48 + tid] = pmu;
      tb[64 + tid] = pa;
      tb[80 + tid] = pbe;
    }
  };
  auto write_x = [&](int chunk, int slot) {
    __bf16 *xi = reinterpret_cast<__bf16 *>(lds + G::OFF_X);
    const float *tb = bnt + slot * 96;
#pragma unroll
    for (int k = 0; k < G::IPT; ++k)
      if (loff[k] >= 0) {
        const int ch = ich[k];
        float v = 0.f;
        if (chunk * G::CK + ch < P.C && goff[k] != kOOB) {
          float xx = st[k];
          if (P.pmean) {
            const float u = (xx - tb[48 + ch]) * tb[64 + ch] + tb[80 + ch];
            xx = u > 0.f ? u : 0.f;
          }
          v = (xx - tb[ch]) * tb[16 + ch] + tb[32 + ch];
          if (P.relu) v = fmaxf(v, 0.f);
        }
        xi[loff[k]] = (__bf16)v;
      }
  };
  // packed W' chunk by LDS-DMA (inline asm: the compiler must not wait for it
  // before unrelated LDS reads); completion by the s_waitcnt before write_x
  const uint64_t wsrc =
      reinterpret_cast<uint64_t>(P.wpk) + (uint64_t)rt * nch * G::W_BYTES;
  const int4f rsw = {(int)(uint32_t)wsrc, (int)((wsrc >> 32) & 0xffff), nch * G::W_BYTES,
                     0x00020000};
  const unsigned ldsw = (unsigned)reinterpret_cast<uintptr_t>(lds + G::OFF_W);
  auto dma_w = [&](int chunk, int buf) {
#pragma unroll
    for (int d = wave; d < 2 * K; d += 4) {
      const unsigned voffw = (unsigned)(chunk * G::W_BYTES + d * 1024 + lane * 16);
      const unsigned m0v = ldsw + (unsigned)(buf * G::W_BYTES + d * 1024);
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
          "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "s"(m0v), "v"(voffw), "s"(rsw)
          : "memory");
    }
  };

  // W' GEMM fragments: wave w -> rows (w&1)*32.., column tiles (w>>1)*4..+3
  const int mi = wave & 1, nj0 = (wave >> 1) * 4;
  const int ao = (hi * 64 + mi * 32 + lo) * 16;  // + k * 2 KiB
  int bo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = (nj0 + j) * 32 + lo;
    bo[j] = ((col < G::NCOLS ? col : 0) * G::SLOTS + hi) * 16;  // + k * 32
  }
  floatx16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  bn_table(0, 0);
  dma_w(0, 0);
  load_x(0);
  spf_wait_all(st);
  __syncthreads();  // BN table, A planes, X pads
  write_x(0, 0);
  for (int c = 0; c < nch; ++c) {
    __syncthreads();  // A: X(c) and W'(c) are in LDS; every wave is done with G(c-1)
    const bool more = c + 1 < nch;
    if (more) {
      bn_table(c + 1, (c + 1) & 1);
      dma_w(c + 1, (c + 1) & 1);
      load_x(c + 1);
    }
    // -- joint contraction on MFMA: G tiles -> bf16 G image
    {
      const char *xi = lds + G::OFF_X;
      const char *ah = lds + G::OFF_AH, *am = lds + G::OFF_AM;
      char *gi = lds + G::OFF_G;
      for (int tt = wave; tt < G::GT; tt += 4) {
        const int grt = tt / G::GC, gct = tt - grt * G::GC;
        floatx16 ga;
#pragma unroll
        for (int i = 0; i < 16; ++i) ga[i] = 0.f;
        const int xo = ((grt * 32 + lo) * G::XP + 8 * hi) * 2;
        const int bo2 = ((gct * 32 + lo) * G::XP + 8 * hi) * 2;
#pragma unroll
        for (int s = 0; s < G::KS; ++s) {
          const bf16x8f a = *reinterpret_cast<const bf16x8f *>(xi + xo + s * 32);
          const bf16x8f bh = *reinterpret_cast<const bf16x8f *>(ah + bo2 + s * 32);
          const bf16x8f bm = *reinterpret_cast<const bf16x8f *>(am + bo2 + s * 32);
          ga = mfma_bf(a, bh, ga);
          ga = mfma_bf(a, bm, ga);
        }
        const int col = gct * 32 + lo;
        const int kk = col / V, v = col - kk * V;
        if (col < G::NGC) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // register group: 4 consecutive channels
            const int row = grt * 32 + 8 * q + 4 * hi;
            const int t = row >> 4, ch0 = row & 15;
            if (t < G::FT) {
              uint2 d;
              d.x = pkbf(ga[4 * q], ga[4 * q + 1]);
              d.y = pkbf(ga[4 * q + 2], ga[4 * q + 3]);
              *reinterpret_cast<uint2 *>(gi + ((t * V + v) * G::SLOTS) * 16 +
                                         (kk * 16 + ch0) * 2) = d;
            }
          }
        }
      }
    }
    __syncthreads();  // B: G(c) complete; X(c) no longer read
    if (P.Gk && rt == 0) {
      // kept G for the backward: item (octet o of the 16K channels, 8-position
      // block b): 8 x ds_read_b128, 8x8 bf16 transpose, 8 x 16-byte stores
      const char *gi = lds + G::OFF_G;
      const int o = tid >> 5, b = tid & 31;
      if (o < 2 * K) {
        unsigned short vv[8][8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int pos = b * 8 + u;
          uint4 r = make_uint4(0u, 0u, 0u, 0u);
          if (pos < G::NCOLS) r = *reinterpret_cast<const uint4 *>(gi + (pos * G::SLOTS + o) * 16);
          const unsigned w4[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) vv[e][u] = (unsigned short)(w4[e >> 1] >> (16 * (e & 1)));
        }
        const int kk = o >> 1;  // partition
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int ch = (o & 1) * 8 + e;
          const int ci = c * G::CK + ch;
          if (ci < P.C) {
            uint4 w;
            w.x = vv[e][0] | ((unsigned)vv[e][1] << 16);
            w.y = vv[e][2] | ((unsigned)vv[e][3] << 16);
            w.z = vv[e][4] | ((unsigned)vv[e][5] << 16);
            w.w = vv[e][6] | ((unsigned)vv[e][7] << 16);
            const int64_t row = (int64_t)n * K * P.C + (int64_t)kk * P.C + ci;
            *reinterpret_cast<uint4 *>(P.Gk + (row * p.n_mtiles + mt) * 256 + b * 8) = w;
          }
        }
      }
    }
    // -- the W' GEMM: K k-steps (one per partition) of 16 channels
    {
      const char *wa = lds + G::OFF_W + (c & 1) * G::W_BYTES + ao;
      const char *gi = lds + G::OFF_G;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const bf16x8f a = *reinterpret_cast<const bf16x8f *>(wa + k * 2048);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x8f b = *reinterpret_cast<const bf16x8f *>(gi + bo[j] + k * 32);
          acc[j] = mfma_bf(a, b, acc[j]);
        }
      }
    }
    if (more) {
      spf_wait_all(st);  // x(c+1) and W'(c+1) landed
      write_x(c + 1, (c + 1) & 1);
    }
  }
  __syncthreads();  // every wave is done with the images (the epilogue reuses LDS)
  conv_tile_epilogue<V, G::NCOLS, true, true>(p, acc, n, r0, m0, smem);
}

// ---------------------------------------------------------------------------
// k_sp_fwd_wide<V, K, ROWS>: the same fused SpatialConv forward for the wide
// two-person graph (V = 50, K = 3; BASELINE cfg5) with ALL output channels in
// one workgroup (ROWS = C_out rounded to 64, <= 256), so the joint contraction
// of a 16-channel chunk -- 3 x 5 tiles x 4 k-steps x 2 A planes, 2.5x the W'
// GEMM's MFMAs at C_out = 64 -- runs once per (clip, frame tile) instead of
// once per 64-row tile. 8 waves (two per SIMD), one workgroup per CU:
//   joint contraction: tile tt of the chunk's RT x GC G tiles -> wave tt % 8;
//   W' GEMM: wave w -> rows (w & 1) * ROWS/2 .. (ROWS/64 32-row blocks) x
//            column tiles 2 (w >> 1), +1; packed bf16 W' [chunk][k][octet]
//            [ROWS][8] by 16-byte LDS-DMA, double-buffered;
//   epilogue: the row-major LDS image epilogue (conv_tile_store_rows) for
//            ROWS <= 128; per-wave register stores at 256 (no BN statistics:
//            residual blocks stay at ROWS <= 128).
// The x chunk of the next step is loaded under this chunk's MFMAs.
// ---------------------------------------------------------------------------
template <int V, int K, int ROWS>
struct SpWideGeo {
  static constexpr int NT = 512;
  static constexpr int FT = kTileCols / V;
  static constexpr int NCOLS = FT * V;
  static constexpr int CK = 16;
  static constexpr int XROWS = CK * FT;
  static constexpr int RT = (XROWS + 31) / 32;
  static constexpr int KW = (V + 15) & ~15;
  static constexpr int KS = KW / 16;
  static constexpr int XP = KW + 8;
  static constexpr int NGC = K * V;
  static constexpr int GC = (NGC + 31) / 32;
  static constexpr int GT = RT * GC;
  static constexpr int SLOTS = 2 * K + 1;
  static constexpr int MB = ROWS / 64;            // 32-row blocks per wave
  static constexpr int X_BYTES = RT * 32 * XP * 2;
  static constexpr int A_BYTES = GC * 32 * XP * 2;
  static constexpr int G_BYTES = NCOLS * SLOTS * 16;
  static constexpr int W_BYTES = K * 2 * ROWS * 16;  // packed W' chunk
  static constexpr int NIT = CK * NCOLS;
  static constexpr int IPT = (NIT + NT - 1) / NT;
  static constexpr int A_IMG = (2 * A_BYTES + 1023) & ~1023;  // both planes, whole KiB
  static constexpr int OFF_AH = 0, OFF_AM = A_BYTES, OFF_X = A_IMG;
  static constexpr int OFF_G = OFF_X + X_BYTES, OFF_W = OFF_G + G_BYTES;
  static constexpr int OFF_BN = OFF_W + 2 * W_BYTES;
  static constexpr int MAIN = OFF_BN + 2 * 6 * 16 * 4;
  static constexpr int EROWS = ROWS < 128 ? ROWS : 128;  // LDS-image epilogue rows
  static constexpr int EPI = ROWS == 256 ? 0 : (EROWS * kEpiPitch + EROWS * V) * 4;
  static constexpr int LDS = MAIN > EPI ? MAIN : EPI;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(IPT == 8, "staging register count");
  static_assert(ROWS == 64 || ROWS == 128 || ROWS == 256, "row tiles");
};

template <int V, int K, int ROWS>
__global__ __launch_bounds__(512, 1) void k_sp_fwd_wide(SpFwdParams P) {
  using G = SpWideGeo<V, K, ROWS>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const ConvGemmParams &p = P.ep;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid % p.n_mtiles;
  const int n = bid / p.n_mtiles;
  const int m0 = mt * G::FT;
  const int TV = P.T * V;
  const int nch = P.nchunks;

  // ---- prologue: A planes (h, m) by 16-byte LDS-DMA of the prebuilt image
  // (k_pack_sp_a), zeroed X pads; landed by the vmcnt(0) before the first barrier
  {
    const __amdgpu_buffer_rsrc_t ra =
        make_rsrc(reinterpret_cast<const float *>(P.aimg), G::A_IMG / 4);
    for (int i = wave; i < G::A_IMG / 1024; i += 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, smem + i * 256, 16,
                                               (unsigned)(i * 1024 + lane * 16), 0, 0, 0);
    unsigned *xz = reinterpret_cast<unsigned *>(lds + G::OFF_X);
    for (int e = tid; e < G::X_BYTES / 4; e += G::NT) xz[e] = 0u;
  }
  // ---- x staging: items (ch, pos), consecutive threads = consecutive positions
  // (item indices recomputed at use: constant divisions, no index registers)
  const uint64_t xsrc = reinterpret_cast<uint64_t>(P.x + (int64_t)n * P.C * TV);
  const int pos_lim = min(G::NCOLS, TV - m0 * V);  // valid positions of the tile
  float st[G::IPT];
  auto load_x = [&](int chunk) {
    const int64_t rem = (int64_t)(P.C - chunk * G::CK) * TV * 4;
    const uint64_t src = xsrc + (uint64_t)chunk * G::CK * TV * 4;
    const int4f rs = {(int)(uint32_t)src, (int)((src >> 32) & 0xffff),
                      (int)(rem > 0x7fffffff ? 0x7fffffff : (rem > 0 ? rem : 0)), 0x00020000};
    unsigned goff[G::IPT];
#pragma unroll
    for (int k = 0; k < G::IPT; ++k) {
      const int e = k * G::NT + tid;
      const int ch = e / G::NCOLS, pos = e - ch * G::NCOLS;
      goff[k] = (e < G::NIT && pos < pos_lim) ? (unsigned)((ch * TV + m0 * V + pos) * 4) : kOOB;
    }
    asm volatile("s_nop 4" ::: "memory");
#pragma unroll
    for (int k = 0; k < G::IPT; ++k)
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen"
                   : "=v"(st[k])
                   : "v"(goff[k]), "s"(rs)
                   : "memory");
  };
  auto wait_x = [&]() {
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(st[0]), "+v"(st[1]), "+v"(st[2]), "+v"(st[3]), "+v"(st[4]), "+v"(st[5]),
                   "+v"(st[6]), "+v"(st[7])::"memory");
  };
  float *bnt = reinterpret_cast<float *>(lds + G::OFF_BN);  // [2][6][16]: mean, a, beta; prev
  auto bn_table = [&](int chunk, int slot) {
    if (tid < 16) {
      const int c = chunk * G::CK + tid;
      float mu = 0.f, a = 0.f, be = 0.f, pmu = 0.f, pa = 0.f, pbe = 0.f;
      if (c < P.C) {
        mu = P.mean[c];
        a = P.invstd[c] * P.g[c];
        be = P.b[c];
        if (P.pmean) {
          pmu = P.pmean[c];
          pa = P.pinvstd[c] * P.pg[c];
          pbe = P.pb[c];
        }
      }
      float *tb = bnt + slot * 96;
      tb[tid] = mu;
      tb[16 + tid] = a;
      tb[32 + tid] = be;
      tb[48 + tid] = pmu;
      tb[64 + tid] = pa;
      tb[80 + tid] = pbe;
    }
  };
  auto write_x = [&](int chunk, int slot) {
    __bf16 *xi = reinterpret_cast<__bf16 *>(lds + G::OFF_X);
    const float *tb = bnt + slot * 96;
#pragma unroll
    for (int k = 0; k < G::IPT; ++k) {
      const int e = k * G::NT + tid;
      const int ch = e / G::NCOLS, pos = e - ch * G::NCOLS;
      const int t = pos / V, w = pos - t * V;
      if (e < G::NIT) {
        float v = 0.f;
        if (chunk * G::CK + ch < P.C && pos < pos_lim) {
          float xx = st[k];
          if (P.pmean) {
            const float u = (xx - tb[48 + ch]) * tb[64 + ch] + tb[80 + ch];
            xx = u > 0.f ? u : 0.f;
          }
          v = (xx - tb[ch]) * tb[16 + ch] + tb[32 + ch];
          if (P.relu) v = fmaxf(v, 0.f);
        }
        xi[(t * 16 + ch) * G::XP + w] = (__bf16)v;
      }
    }
  };
  const uint64_t wsrc = reinterpret_cast<uint64_t>(P.wpk);
  const int4f rsw = {(int)(uint32_t)wsrc, (int)((wsrc >> 32) & 0xffff), nch * G::W_BYTES,
                     0x00020000};
  const unsigned ldsw = (unsigned)reinterpret_cast<uintptr_t>(lds + G::OFF_W);
  auto dma_w = [&](int chunk, int buf) {
#pragma unroll
    for (int d = wave; d < G::W_BYTES / 1024; d += 8) {
      const unsigned voffw = (unsigned)(chunk * G::W_BYTES + d * 1024 + lane * 16);
      const unsigned m0v = ldsw + (unsigned)(buf * G::W_BYTES + d * 1024);
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
          "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "s"(m0v), "v"(voffw), "s"(rsw)
          : "memory");
    }
  };

  // W' GEMM: wave w -> rows mi*ROWS/2 + rb*32 (rb < MB), column tiles cj*2 + j
  const int mi = wave & 1, cj = wave >> 1;
  int ao[G::MB];
#pragma unroll
  for (int rb = 0; rb < G::MB; ++rb) ao[rb] = (hi * ROWS + mi * (ROWS / 2) + rb * 32 + lo) * 16;
  int bo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (cj * 2 + j) * 32 + lo;
    bo[j] = ((col < G::NCOLS ? col : 0) * G::SLOTS + hi) * 16;
  }
  floatx16 acc[G::MB][2];
#pragma unroll
  for (int rb = 0; rb < G::MB; ++rb)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[rb][j][i] = 0.f;

  bn_table(0, 0);
  dma_w(0, 0);
  load_x(0);
  wait_x();
  __syncthreads();  // BN table, A planes, X pads
  write_x(0, 0);
  for (int c = 0; c < nch; ++c) {
    __syncthreads();  // A: X(c) and W'(c) are in LDS; every wave is done with G(c-1)
    const bool more = c + 1 < nch;
    if (more) {
      bn_table(c + 1, (c + 1) & 1);
      dma_w(c + 1, (c + 1) & 1);
      load_x(c + 1);
    }
    // -- joint contraction on MFMA: G tiles -> bf16 G image
    {
      const char *xi = lds + G::OFF_X;
      const char *ah = lds + G::OFF_AH, *am = lds + G::OFF_AM;
      char *gi = lds + G::OFF_G;
      for (int tt = wave; tt < G::GT; tt += 8) {
        const int grt = tt / G::GC, gct = tt - grt * G::GC;
        floatx16 ga;
#pragma unroll
        for (int i = 0; i < 16; ++i) ga[i] = 0.f;
        const int xo = ((grt * 32 + lo) * G::XP + 8 * hi) * 2;
        const int bo2 = ((gct * 32 + lo) * G::XP + 8 * hi) * 2;
#pragma unroll
        for (int s = 0; s < G::KS; ++s) {
          const bf16x8f xa = *reinterpret_cast<const bf16x8f *>(xi + xo + s * 32);
          const bf16x8f bh = *reinterpret_cast<const bf16x8f *>(ah + bo2 + s * 32);
          const bf16x8f bm = *reinterpret_cast<const bf16x8f *>(am + bo2 + s * 32);
          ga = mfma_bf(xa, bh, ga);
          ga = mfma_bf(xa, bm, ga);
        }
        const int col = gct * 32 + lo;
        const int kk = col / V, v = col - kk * V;
        if (col < G::NGC) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // register group: 4 consecutive channels
            const int row = grt * 32 + 8 * q + 4 * hi;
            const int t = row >> 4, ch0 = row & 15;
            if (t < G::FT) {
              uint2 d;
              d.x = pkbf(ga[4 * q], ga[4 * q + 1]);
              d.y = pkbf(ga[4 * q + 2], ga[4 * q + 3]);
              *reinterpret_cast<uint2 *>(gi + ((t * V + v) * G::SLOTS) * 16 + (kk * 16 + ch0) * 2) =
                  d;
            }
          }
        }
      }
    }
    __syncthreads();  // B: G(c) complete; X(c) no longer read
    // -- the W' GEMM: K k-steps (one per partition) of 16 channels
    {
      const char *wa = lds + G::OFF_W + (c & 1) * G::W_BYTES;
      const char *gi = lds + G::OFF_G;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        bf16x8f a[G::MB], b[2];
#pragma unroll
        for (int rb = 0; rb < G::MB; ++rb)
          a[rb] = *reinterpret_cast<const bf16x8f *>(wa + k * 2 * ROWS * 16 + ao[rb]);
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const bf16x8f *>(gi + bo[j] + k * 32);
#pragma unroll
        for (int rb = 0; rb < G::MB; ++rb)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[rb][j] = mfma_bf(a[rb], b[j], acc[rb][j]);
      }
    }
    if (more) {
      wait_x();  // x(c+1) and W'(c+1) landed
      write_x(c + 1, (c + 1) & 1);
    }
    if (P.Gk) {
      // kept G for the backward dW' (k_wgrad_gemm_gk layout Gk[n][k*C_in + ci]
      // [mtile][256]), from the LDS image after the x wait, so the stores drain
      // under the next chunk: item (position, octet) = 8 channels of one
      // position; lanes = consecutive positions (128-byte pieces per store);
      // the 256 - NCOLS pad positions are written as zeros
      const char *gi = lds + G::OFF_G;
      for (int e = tid; e < 256 * 2 * K; e += G::NT) {
        const int o = e >> 8, pos = e & 255;
        uint4 r = make_uint4(0u, 0u, 0u, 0u);
        if (pos < G::NCOLS) r = *reinterpret_cast<const uint4 *>(gi + (pos * G::SLOTS + o) * 16);
        const unsigned w4[4] = {r.x, r.y, r.z, r.w};
        const int kk = o >> 1;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int ci = c * G::CK + (o & 1) * 8 + q;
          if (ci < P.C) {
            const int64_t grow = ((int64_t)n * K + kk) * P.C + ci;
            P.Gk[(grow * p.n_mtiles + mt) * 256 + pos] =
                __builtin_bit_cast(__bf16, (unsigned short)(w4[q >> 1] >> (16 * (q & 1))));
          }
        }
      }
    }
  }
  if constexpr (ROWS == 256) {
    // ---- epilogue, 256 rows: each wave stores its own tiles from registers
    // (an LDS image of all rows does not fit; bias table, no statistics: the
    // launcher keeps residual blocks, whose BN2 statistics come from here, at
    // ROWS <= 128). Lanes = consecutive positions: 128-byte row pieces.
    const __amdgpu_buffer_rsrc_t rs_o =
        p.out_bf16 ? make_rsrc(reinterpret_cast<const float *>(reinterpret_cast<const __bf16 *>(p.out) +
                                                               (int64_t)n * p.out_bstride),
                               (p.out_bstride + 1) / 2)
                   : make_rsrc(p.out + (int64_t)n * p.out_bstride, p.out_bstride);
    const __amdgpu_buffer_rsrc_t rs_bv = make_rsrc(p.bias_rv, (int64_t)p.R * V);
    const int ostride = p.T_dst * V;
    // (bias-table loads one register group ahead of its stores: vmcnt counts loads
    // and stores in one in-order counter, so a load issued after a store is only
    // waited for together with that store -- one store latency per element)
    constexpr int NGRP = 2 * G::MB;  // (column tile j, row block rb) groups of 16
    auto bias16 = [&](int gidx, float (&bv)[16]) {
      const int j = gidx / G::MB, rb = gidx % G::MB;
      const int col = (cj * 2 + j) * 32 + lo;
      const bool cok = col < pos_lim;
      const int v = col % V;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = mi * (ROWS / 2) + rb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
        const bool ok = cok && row < p.R;
        bv[i] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rs_bv, ok ? (row * V + v) * 4 : (int)kOOB,
                                                        0, 0));
      }
    };
    float bvb[2][16];
    bias16(0, bvb[0]);
#pragma unroll
    for (int gidx = 0; gidx < NGRP; ++gidx) {
      if (gidx + 1 < NGRP) bias16(gidx + 1, bvb[(gidx + 1) & 1]);
      const int j = gidx / G::MB, rb = gidx % G::MB;
      const int col = (cj * 2 + j) * 32 + lo;
      const bool cok = col < pos_lim;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = mi * (ROWS / 2) + rb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
        const bool ok = cok && row < p.R;
        const float val = acc[rb][j][i] + bvb[gidx & 1][i];
        const int e = row * ostride + m0 * V + col;
        if (p.out_bf16)
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (__bf16)val),
                                                rs_o, ok ? e * 2 : (int)kOOB, 0, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, val), rs_o,
                                                ok ? e * 4 : (int)kOOB, 0, 0);
      }
    }
    return;
  } else {
    // ---- epilogue: row-major LDS image (conv_tile_store_rows), one pass
    __syncthreads();  // every wave is done with the images
#pragma unroll
    for (int rb = 0; rb < G::MB; ++rb)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc_to_img(smem, acc[rb][j], mi * (ROWS / 2) + rb * 32, (cj * 2 + j) * 32);
    __syncthreads();
    conv_tile_store_rows<V, G::NCOLS, G::NT, ROWS, true, true>(p, smem, smem + ROWS * kEpiPitch, n, 0,
                                                         m0);
  }
}

// W (K*C_out, C_in) -> wpk[rt][chunk][k][octet][rows][8] bf16 (zero padded;
// rows = 64 per row tile, or all ROWS of k_sp_fwd_wide)
__global__ void k_pack_sp_w_bf16(const float *W, __bf16 *wpk, int K, int R, int C, int nch,
                                 int rows, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int j = (int)(idx & 7);
  int64_t t = idx >> 3;
  const int rl = (int)(t % rows);
  t /= rows;
  const int o = (int)(t & 1);
  t >>= 1;
  const int k = (int)(t % K);
  t /= K;
  const int chunk = (int)(t % nch);
  const int rt = (int)(t / nch);
  const int r = rt * rows + rl, c = chunk * 16 + o * 8 + j;
  float v = 0.f;
  if (r < R && c < C) v = W[((int64_t)k * R + r) * C + c];
  wpk[idx] = (__bf16)v;
}

// A (K, V, V) -> the LDS image of both kernels: planes h, m of the gather's B
// operand [c = k*V + v][w] (pitch XP bf16, zero padded), whole KiB
__global__ void k_pack_sp_a(const float *A, __bf16 *img, int K, int V, int GC, int XP,
                            int plane, int total) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int pl = e / plane, r = e - pl * plane;
  float a = 0.f;
  if (pl < 2) {
    const int c = r / XP, w = r - c * XP;
    if (c < K * V && w < V) a = A[c * V + w];
  }
  const __bf16 h = (__bf16)a;
  img[e] = pl == 0 ? h : (pl == 1 ? (__bf16)(a - (float)h) : (__bf16)0.f);
}

bool sp_fwd_bf16_supported(int C, int V, int K, int R, bool residual) {
  if (C < 16) return false;  // the first block's 3-channel input stays on the fp32 path
  if (K < 1 || K > 3) return false;
  if (V == 18 || V == 25) return true;
  // the two-person graph: all output channels in one workgroup (k_sp_fwd_wide;
  // its 256-row epilogue computes no BN2 statistics for the residual block)
  return V == 50 && K == 3 && (R <= 128 || (R <= 256 && !residual));
}

size_t sp_fwd_bf16_wpk_bytes(int C, int R, int K, int V) {
  const int KW = (V + 15) & ~15, XP = KW + 8, GC = (K * V + 31) / 32;
  const size_t a = ((size_t)2 * GC * 32 * XP * 2 + 1023) & ~(size_t)1023;
  const size_t w = (size_t)((R + 255) / 64) * ((C + 15) / 16) * K * 2 * 64 * 8 * 2;  // rows <= 256
  return ((w + 1023) & ~(size_t)1023) + a;
}

size_t sp_keep_g_bytes(int N, int C, int T, int V, int K) {
  const int FT = kTileCols / V;
  return (size_t)N * K * C * ((T + FT - 1) / FT) * 256 * 2;
}

template <int V, int K>
static void launch_spf(const SpFwdParams &P, int nblk, hipStream_t s) {
  constexpr int lds = SpFwdGeo<V, K>::LDS;
  hipLaunchKernelGGL((k_sp_fwd_bf16<V, K>), dim3(nblk), dim3(256), lds, s, P);
}

template <int V, int K, int ROWS>
static void launch_spw(const SpFwdParams &P, int nblk, hipStream_t s) {
  constexpr int lds = SpWideGeo<V, K, ROWS>::LDS;
  hipLaunchKernelGGL((k_sp_fwd_wide<V, K, ROWS>), dim3(nblk), dim3(512), lds, s, P);
}

hipError_t launch_sp_fwd_bf16(const float *x, const float *mean, const float *invstd,
                              const float *g, const float *b, const float *A, const float *W,
                              const float *biasZ, void *wpk, float *Z, int z_bf16, __bf16 *Gk,
                              double *ssum,
                              double *ssq, int N, int C, int R, int T, int V, int K, int relu,
                              hipStream_t s, const PrevBn *prev) {
  if (!sp_fwd_bf16_supported(C, V, K, R, relu != 0)) return hipErrorInvalidValue;
  // all output channels per workgroup: the two-person graph, and V = 25 with
  // K = 3 (STGCN_AB_SPF_NARROW25 build: the 64-row k_sp_fwd_bf16 there, A/B only)
  constexpr bool narrow25 = STGCN_AB_SPF_NARROW25 != 0;
  const bool wide = V == 50 || (V == 25 && K == 3 && !narrow25 && (R <= 128 || !relu));
  const int nch = (C + 15) / 16;
  const int rows = !wide ? 64 : (R <= 64 ? 64 : (R <= 128 ? 128 : 256));
  const int nrt = (R + rows - 1) / rows;
  {
    const int64_t total = (int64_t)nrt * nch * K * 2 * rows * 8;
    hipLaunchKernelGGL(k_pack_sp_w_bf16, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, W,
                       reinterpret_cast<__bf16 *>(wpk), K, R, C, nch, rows, total);
  }
  // the A image after the packed W' in the scratch
  const size_t wbytes = ((size_t)nrt * nch * K * 2 * rows * 8 * 2 + 1023) & ~(size_t)1023;
  __bf16 *aimg = reinterpret_cast<__bf16 *>(reinterpret_cast<char *>(wpk) + wbytes);
  {
    const int KW = (V + 15) & ~15, XP = KW + 8, GC = (K * V + 31) / 32;
    const int plane = GC * 32 * XP;
    const int total = (2 * plane * 2 + 1023) / 1024 * 1024 / 2;  // bf16 elements, whole KiB
    hipLaunchKernelGGL(k_pack_sp_a, dim3((total + 255) / 256), dim3(256), 0, s, A, aimg, K, V, GC,
                       XP, plane, total);
  }
  SpFwdParams P{};
  P.aimg = aimg;
  P.x = x;
  P.mean = mean;
  P.invstd = invstd;
  P.g = g;
  P.b = b;
  P.A = A;
  if (prev && prev->mean) {
    P.pmean = prev->mean;
    P.pinvstd = prev->invstd;
    P.pg = prev->g;
    P.pb = prev->b;
  }
  P.wpk = reinterpret_cast<const __bf16 *>(wpk);
  P.Gk = Gk;
  P.C = C;
  P.T = T;
  P.relu = relu;
  P.nchunks = nch;
  ConvGemmParams &p = P.ep;
  p.out = Z;
  p.out_bf16 = z_bf16;
  p.bias_rv = biasZ;
  p.stat_sum = ssum;
  p.stat_sq = ssq;
  p.out_bstride = (int64_t)R * T * V;
  p.R = R;
  p.V = V;
  p.FT = kTileCols / V;
  p.M = T;
  p.T_dst = T;
  p.s_out = 1;
  p.p_out = 0;
  p.N = N;
  p.n_mtiles = (T + p.FT - 1) / p.FT;
  p.n_rtiles = nrt;
  const int nblk = N * p.n_mtiles * nrt;
  if (wide && V == 50) {
    if (rows == 64) launch_spw<50, 3, 64>(P, nblk, s);
    else if (rows == 128) launch_spw<50, 3, 128>(P, nblk, s);
    else launch_spw<50, 3, 256>(P, nblk, s);
    return hipGetLastError();
  }
  if (wide) {
    if (rows == 64) launch_spw<25, 3, 64>(P, nblk, s);
    else if (rows == 128) launch_spw<25, 3, 128>(P, nblk, s);
    else launch_spw<25, 3, 256>(P, nblk, s);
    return hipGetLastError();
  }
#define SPF_K(VV)                            \
  if (K == 1) launch_spf<VV, 1>(P, nblk, s); \
  else if (K == 2) launch_spf<VV, 2>(P, nblk, s); \
  else launch_spf<VV, 3>(P, nblk, s);
  if (V == 18) {
    SPF_K(18)
  } else {
    SPF_K(25)
  }
#undef SPF_K
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_wgrad_gemm_gk<TR>: the spatial weight gradient dW' = dZ G^T of the bf16
// path reading the G kept by k_sp_fwd_bf16 (bf16, Gk[n][c][mtile][256]):
//   slab[split][r][c] = sum_{items} sum_{i < 32} dZ[n][r][m0*V + kc*32 + i]
//                                               * Gk[n][c][mt][kc*32 + i]
// item = (clip n, frame tile mt, 32-position piece kc < 8). Tiles TR x 256
// (8 or 4 waves of 64 x 64) as k_wgrad_gemm_bf16; dZ staged in fp32 by 4-byte
// LDS-DMA and rounded at fragment read, G staged in bf16 by 16-byte LDS-DMA
// into rows of 5 slots (the fifth an OOB zero pad: 80-byte pitch, conflict-free
// ds_read_b128 straight into the MFMA B fragment, no conversion).
// Staging runs through an NS-slot LDS ring: items it+1 .. it+NS-2 stay in
// flight while item it computes; each wave waits only for its own DMAs of item
// it (vmcnt retires loads in order) and one barrier publishes the item (a
// fenced __syncthreads would drain the ring). The item's fragments are read
// first as 16-byte vectors (one LDS wait), then converted and multiplied.
// PB: dZ is stored in bf16 (capi.hip dz_bf16): staged as bf16 PAIRS by 4-byte
// LDS-DMA (a row's piece from the even element at or below its start: rows
// of an odd-length clip row start at odd elements on odd rows), rows of 20
// dwords (17 used, 80-byte pitch); a fragment = one ds_read_b128 + one
// ds_read_b32, shifted by 16 bits on odd-start rows, positions past the piece
// masked to 0 -- the same bf16 operand values as rounding the fp32 dZ at
// fragment read.
// ---------------------------------------------------------------------------
template <int TR, bool PB = false>
struct WgGkGeo {
  static constexpr int TC = 256, KC = 32;
  static constexpr int PITCH = PB ? 20 : KC + 4;            // P pitch (dwords)
  static constexpr int PUSED = KC / 2 + 1;                  // (PB) pairs staged per row
  static constexpr int PSZ = TR * PITCH;                    // dwords
  static constexpr int QSLOTS = TC * 5;                     // 16-byte slots of the G image
  static constexpr int QBYTES = QSLOTS * 16;
  static constexpr int PBYTES = PSZ * 4;
  static constexpr int BUF = PBYTES + QBYTES;               // bytes per buffer
  static constexpr int NWR = TR / 64, NW = NWR * 4, NTH = NW * 64;
  static constexpr int PROUNDS = (PSZ + NTH - 1) / NTH;
  static constexpr int QROUNDS = (QSLOTS + NTH - 1) / NTH;
  // LDS-DMAs every wave issues per item (the P rounds are whole; a partial last
  // Q round adds one on the first waves only): the ring's vmcnt allowance per
  // item still in flight (a wave issuing more waits slightly more, never less)
  static constexpr int DMIN = PROUNDS + QSLOTS / NTH;
  static_assert(PSZ % NTH == 0, "whole P rounds");
};

// s_waitcnt vmcnt(ahead * D) (immediates only), then one unfenced barrier
template <int D>
__device__ __forceinline__ void gk_ring_wait(int ahead) {
  static_assert(2 * D < 64, "vmcnt range");
  if (ahead >= 2)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(2 * D) : "memory");
  else if (ahead == 1)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(D) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int TR, int NS, bool PB>
__global__ __launch_bounds__(512, 1) void k_wgrad_gemm_gk(WgradParams p) {
  using G = WgGkGeo<TR, PB>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = p.n_rtiles * p.n_jtiles;
  const int tile = bid % ntiles;
  const int split = bid / ntiles;
  const int ct = tile % p.n_jtiles, rt = tile / p.n_jtiles;
  const int V = p.V, L = p.M * V, FTV = (kTileCols / V) * V;
  const int nmt = p.n_mtiles / 8;  // frame tiles per clip
  const int r0 = rt * TR, c0 = ct * G::TC;
  const int prow_lim = min(TR, p.R - r0), qrow_lim = min(G::TC, p.C - c0);
  const int total = p.N * p.n_mtiles;
  const int per = (total + p.S - 1) / p.S;
  const int it0 = split * per, it1 = min(total, it0 + per);
  // P: round i of this wave fills floats [(i*NW + wave)*64 + lane]
  int prow[G::PROUNDS], pcol[G::PROUNDS];
#pragma unroll
  for (int i = 0; i < G::PROUNDS; ++i) {
    const int pos = (i * G::NW + wave) * 64 + lane;
    prow[i] = pos < G::PSZ ? pos / G::PITCH : -1;
    pcol[i] = pos < G::PSZ ? pos - prow[i] * G::PITCH : 0;
  }
  // Q: round i fills slots [(i*NW + wave)*64 + lane]: row = slot / 5, piece = slot % 5
  int qrow[G::QROUNDS], qpc[G::QROUNDS];
#pragma unroll
  for (int i = 0; i < G::QROUNDS; ++i) {
    const int sl = (i * G::NW + wave) * 64 + lane;
    qrow[i] = sl < G::QSLOTS ? sl / 5 : -1;
    qpc[i] = sl < G::QSLOTS ? sl - (sl / 5) * 5 : 4;
  }
  const __bf16 *Gk = reinterpret_cast<const __bf16 *>(p.Q);
  auto stage = [&](int it, char *buf) {
    const int n = it / p.n_mtiles, rem = it - n * p.n_mtiles;
    const int mt = rem >> 3, kc = rem & 7;
    const int l0 = mt * FTV + kc * G::KC;
    const int lim = min(min(G::KC, FTV - kc * G::KC), L - l0);  // valid positions of the piece
    // (PB: a resource over the bf16 tensor, in fp32 units of its bytes; r0 and the
    // clip stride are even, so pair boundaries are dword boundaries)
    const __amdgpu_buffer_rsrc_t rs_p =
        PB ? make_rsrc(reinterpret_cast<const float *>(reinterpret_cast<const __bf16 *>(p.P) +
                                                       (int64_t)n * p.p_bstride + (int64_t)r0 * L),
                       ((int64_t)prow_lim * L + 1) / 2)
           : make_rsrc(p.P + (int64_t)n * p.p_bstride + (int64_t)r0 * L, (int64_t)prow_lim * L);
#pragma unroll
    for (int i = 0; i < G::PROUNDS; ++i) {
      const int base = (i * G::NW + wave) * 64;  // wave-uniform
      if (base < G::PSZ) {
        unsigned voff;
        if constexpr (PB) {  // pair pcol of the row's piece, from element (row start - sh)
          const int sh = (prow[i] & 1) & (L & 1);
          const int e = 2 * pcol[i] - sh;  // first element of the pair, rel. to the piece
          const bool ok = prow[i] >= 0 && prow[i] < prow_lim && pcol[i] < G::PUSED && e < lim;
          voff = ok ? (unsigned)(prow[i] * L + l0 + e) * 2u : kOOB;
        } else {
          const bool ok = prow[i] >= 0 && prow[i] < prow_lim && pcol[i] < lim;
          voff = ok ? (unsigned)(prow[i] * L + l0 + pcol[i]) * 4u : kOOB;
        }
        blds_f32(rs_p, voff, reinterpret_cast<float *>(buf) + base);
      }
    }
    // Gk rows of this clip / column tile: (c0 + row) * nmt * 256 + mt * 256 + kc * 32
    const __amdgpu_buffer_rsrc_t rs_q = make_rsrc(
        reinterpret_cast<const float *>(Gk + ((int64_t)n * p.C + c0) * nmt * 256),
        (int64_t)qrow_lim * nmt * 256 / 2);
#pragma unroll
    for (int i = 0; i < G::QROUNDS; ++i) {
      const int base = (i * G::NW + wave) * 64;
      if (base < G::QSLOTS) {
        const bool ok = qrow[i] >= 0 && qrow[i] < qrow_lim && qpc[i] < 4;
        const unsigned voff =
            ok ? (unsigned)((qrow[i] * nmt + mt) * 256 + kc * G::KC + qpc[i] * 8) * 2u : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs_q, reinterpret_cast<float *>(buf + G::PBYTES + base * 16), 16, voff, 0, 0, 0);
      }
    }
  };
  const int wr = wave / 4, wc = wave % 4;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  static_assert(NS >= 2 && NS <= 4, "ring depth");
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (it0 + k < it1) stage(it0 + k, lds + k * G::BUF);
  int sl = 0;  // ring slot of item it
  for (int it = it0; it < it1; ++it) {
    // items it+1 .. it+NS-2 may stay in flight; the barrier also retires every
    // wave's reads of item it-1, whose slot the next staging reuses
    gk_ring_wait<G::DMIN>(min(NS - 2, it1 - 1 - it));
    if (it + NS - 1 < it1) stage(it + NS - 1, lds + (sl == 0 ? NS - 1 : sl - 1) * G::BUF);
    const char *cur = lds + sl * G::BUF;
    sl = sl + 1 == NS ? 0 : sl + 1;
    const float *pa = reinterpret_cast<const float *>(cur) + (wr * 64 + lo) * G::PITCH + 8 * hi;
    // (PB: dword 4 hi of the row = its pairs from element 8 hi - sh; sh = 1 on odd
    // rows of an odd-length clip row; the item's valid positions: lim_b)
    const unsigned *pab = reinterpret_cast<const unsigned *>(cur) + (wr * 64 + lo) * G::PITCH + 4 * hi;
    const bool shb = PB && (lo & 1) && (L & 1);  // rows wr*64 + i*32 + lo: parity of lo
    int lim_b = G::KC;
    if constexpr (PB) {
      const int n_it = it / p.n_mtiles, rem_it = it - n_it * p.n_mtiles;
      const int l0b = (rem_it >> 3) * FTV + (rem_it & 7) * G::KC;
      lim_b = min(min(G::KC, FTV - (rem_it & 7) * G::KC), L - l0b);
    }
    const char *qb = cur + G::PBYTES + ((wc * 64 + lo) * 5 + hi) * 16;
    // every fragment of the item first, as 16-byte reads (rows are 16-byte
    // aligned: PITCH * 4 = 144 B), one LDS wait, then the conversions and the
    // MFMAs (element-wise reads compiled to b96 + b32 pieces, each waited on
    // before its conversion: the loop was LDS-latency bound)
    constexpr int NKS = G::KC / 16;
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    f32x4v pf[NKS][2][2];
    uint4 pq[NKS][2];
    unsigned pe[NKS][2];
    bf16x8f b[NKS][2];
#pragma unroll
    for (int s = 0; s < NKS; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if constexpr (PB) {
          const unsigned *src = pab + i * 32 * G::PITCH + 8 * s;
          pq[s][i] = *reinterpret_cast<const uint4 *>(__builtin_assume_aligned(src, 16));
          pe[s][i] = src[4];
        } else {
          const f32x4v *src = reinterpret_cast<const f32x4v *>(
              __builtin_assume_aligned(pa + i * 32 * G::PITCH + 16 * s, 16));
          pf[s][i][0] = src[0];
          pf[s][i][1] = src[1];
        }
      }
#pragma unroll
    for (int s = 0; s < NKS; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b[s][j] = *reinterpret_cast<const bf16x8f *>(qb + j * 32 * 5 * 16 + s * 32);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      bf16x8f a[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if constexpr (PB) {
          const uint4 q = pq[s][i];
          uint4 w = q;
          if (shb) {  // odd-start row: elements from the high half of dword 0
            w.x = __builtin_amdgcn_alignbit(q.y, q.x, 16);
            w.y = __builtin_amdgcn_alignbit(q.z, q.y, 16);
            w.z = __builtin_amdgcn_alignbit(q.w, q.z, 16);
            w.w = __builtin_amdgcn_alignbit(pe[s][i], q.w, 16);
          }
          // positions k = 16 s + 8 hi + j past the piece (lim_b) are 0 (the pair
          // at the boundary and, on shifted rows, the element after it)
          const int k0 = 16 * s + 8 * hi;
          if (k0 + 8 > lim_b) {
            unsigned m[4];
#pragma unroll
            for (int d = 0; d < 4; ++d)
              m[d] = (k0 + 2 * d < lim_b ? 0xffffu : 0u) | (k0 + 2 * d + 1 < lim_b ? 0xffff0000u : 0u);
            w.x &= m[0];
            w.y &= m[1];
            w.z &= m[2];
            w.w &= m[3];
          }
          a[i] = __builtin_bit_cast(bf16x8f, w);
        } else {
          const f32x4v lo4 = pf[s][i][0], hi4 = pf[s][i][1];
          a[i] = bf16x8f{(__bf16)lo4.x, (__bf16)lo4.y, (__bf16)lo4.z, (__bf16)lo4.w,
                         (__bf16)hi4.x, (__bf16)hi4.y, (__bf16)hi4.z, (__bf16)hi4.w};
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf(a[i], b[s][j], acc[i][j]);
    }
  }
  float *slab = p.slab + (int64_t)split * p.R * p.C;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = c0 + wc * 64 + j * 32 + lo;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = r0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
        if (r < p.R && c < p.C) slab[(int64_t)r * p.C + c] = acc[i][j][e];
      }
    }
}

void plan_wgrad_gk(WgradParams &w, int T) {
  const int FT = kTileCols / w.V;
  w.FT = 0;
  w.CT = w.R > 64 ? 128 : 64;
  w.n_mtiles = (T + FT - 1) / FT * 8;
  w.n_rtiles = (w.R + w.CT - 1) / w.CT;
  w.n_jtiles = (w.C + 255) / 256;
  const int tiles = w.n_rtiles * w.n_jtiles;
  w.S = std::max(1, std::min((256 + tiles - 1) / tiles, w.N * w.n_mtiles));
  w.bf16 = 1;
}

hipError_t launch_wgrad_gk(const WgradParams &p, hipStream_t s) {
  const int nblk = p.n_rtiles * p.n_jtiles * p.S;
  // ring depth 4 (155.6 / 118.8 KiB, one workgroup per CU, three items in
  // flight): cfg3 5289 vs 5155-5187, cfg5 2352 vs 2301-2303 clips/s against 2
  // slots (two workgroups per CU, one item of lookahead each) in one A/B call.
  // (Before the fragment reads were 16-byte vectors the loop was LDS-latency
  // bound and 2 slots won: 5141 vs 5063.) STGCN_AB_GK_SLOTS2 builds: A/B only.
  constexpr bool two = STGCN_AB_GK_SLOTS2 != 0;
  static_assert(4 * WgGkGeo<128>::BUF <= 160 * 1024, "LDS budget");
#define GK_LAUNCH(TR, NS, PB)                                                                \
  hipLaunchKernelGGL((k_wgrad_gemm_gk<TR, NS, PB>), dim3(nblk), dim3((WgGkGeo<TR, PB>::NTH)), \
                     (NS * WgGkGeo<TR, PB>::BUF), s, p)
  if (p.p_bf16) {  // bf16 dZ (capi.hip dz_bf16)
    if (p.CT == 128) GK_LAUNCH(128, 4, true); else GK_LAUNCH(64, 4, true);
  } else if (p.CT == 128) {
    if (two) GK_LAUNCH(128, 2, false); else GK_LAUNCH(128, 4, false);
  } else {
    if (two) GK_LAUNCH(64, 2, false); else GK_LAUNCH(64, 4, false);
  }
#undef GK_LAUNCH
  return hipGetLastError();
}

}  // namespace stgcn

// bf16 GEMM kernels of libstgcn_hip.so (STGCN_F_BF16) — gfx950 only.
//
// The channel contractions of the block (spatial 1x1 conv, (9,1) temporal conv
// forward / data-grad / weight-grad, residual projection) on
// v_mfma_f32_32x32x16_bf16: operands rounded to bf16 (RNE) while they are
// staged into LDS, fp32 accumulation, fp32 tensors in HBM (the block's
// interface and every other kernel stay fp32; the joint contractions with A
// and BatchNorm are fp32 / fp64 as in the fp32 path). This is the "bf16
// channel GEMMs with fp32 accumulate and fp32 A" configuration of
// BASELINE.json cfg3 / cfg5 (SURVEY.md §8c tolerance 2e-2).
//
// Operand fragments of v_mfma_f32_32x32x16_bf16 (lane l, r = l & 31,
// h = l >> 5): A[row r][k = 8h + j], B[k = 8h + j][col r], j = 0..7 — eight
// consecutive k per lane, so each LDS image keeps the reduction index
// innermost: the conv GEMM stages its input window position-major with the
// chunk's channels contiguous ([pos][channel], 16-byte slots, odd slot pitch),
// the weight gradient stages both operands row-major over (frame, joint)
// positions with the joint axis padded to a multiple of 4.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "internal.h"

namespace stgcn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef int int4v __attribute__((ext_vector_type(4)));

// One 4-byte LDS-DMA piece per lane: LDS[lds_wave + 4 lane] = src[voff] (kOOB
// -> 0). Inline asm, so hipcc neither counts it nor waits for it before LDS
// reads of other buffers (the caller waits with an explicit s_waitcnt vmcnt).
__device__ __forceinline__ void dma_b32(int4v rs, unsigned voff, unsigned lds_wave) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
      "buffer_load_dword %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(__builtin_amdgcn_readfirstlane(lds_wave)), "v"(voff), "s"(rs)
      : "memory");
}
// (wave-uniform values the compiler cannot prove uniform, for "s" operands)
__device__ __forceinline__ int4v uniform4(int4v v) {
  return int4v{__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
               __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w)};
}

__device__ __forceinline__ floatx16 mfma_bf16(bf16x8 a, bf16x8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// two floats -> one dword of two bf16 (round to nearest even, v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}

// 4 consecutive bf16 elements starting at element e (stored as bf16; byte offset
// base = 2 e, or kOOB) as two packed dwords: dword loads from the even element at
// or below e, shifted by 16 bits when e is odd (odd V only: then a third dword)
template <bool ODD_POSSIBLE>
__device__ __forceinline__ void ld_b16x4(__amdgpu_buffer_rsrc_t rs, unsigned base, unsigned &x,
                                         unsigned &y) {
  const unsigned b = base == kOOB ? kOOB : (base & ~3u);
  const unsigned d0 = __builtin_amdgcn_raw_buffer_load_b32(rs, b, 0, 0);
  const unsigned d1 = __builtin_amdgcn_raw_buffer_load_b32(rs, b == kOOB ? kOOB : b + 4u, 0, 0);
  if constexpr (ODD_POSSIBLE) {
    const unsigned d2 = __builtin_amdgcn_raw_buffer_load_b32(rs, b == kOOB ? kOOB : b + 8u, 0, 0);
    const bool odd = base != kOOB && (base & 2u);
    x = odd ? __builtin_amdgcn_alignbit(d1, d0, 16) : d0;
    y = odd ? __builtin_amdgcn_alignbit(d2, d1, 16) : d1;
  } else {
    x = d0;
    y = d1;
  }
}
__device__ __forceinline__ float ld_f32(__amdgpu_buffer_rsrc_t rs, unsigned voff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, 0, 0));
}

// ---------------------------------------------------------------------------
// k_conv_bf16: the ConvGemmParams GEMM (see internal.h) on bf16 MFMA.
// Workgroup = 4 waves, tile = 64 rows x FT*V columns (FT = kTileCols / V, the
// fp32 plan), wave w: rows (w&1)*32..+31, column tiles (w>>1)*4..+3.
// k-step = one tap q x 16 channels of the chunk (CK channels per chunk):
//   A fragment: packed weights [q][channel octet][64 rows][8] (one ds_read_b128),
//   B fragment: the input window [position][CK channels] at position
//               colpos + q*V (one ds_read_b128; slot pitch CK/8 + 1 is odd,
//               so any 16 lanes of consecutive positions are conflict-free).
// Staging: the weights (already bf16 in HBM, wpk) move by 16-byte LDS-DMA;
// the window is loaded as fp32 dwords (consecutive lanes = consecutive
// positions of one channel: coalesced), converted, and written as 16-byte
// [position][8 channels] pieces. Two LDS buffers; chunk i+1's loads are in
// flight under chunk i's MFMAs; one barrier per chunk.
// ---------------------------------------------------------------------------
template <int NQ, int CK, int V, int SIN>
struct ConvBf16Geo {
  static constexpr int FT = kTileCols / V;
  static constexpr int NCOLS = FT * V;
  static constexpr int SPAN = (SIN * (FT - 1) + NQ) * V;  // window positions
  static constexpr int OCT = CK / 8;                      // channel octets per position
  static constexpr int SLOTS = OCT + 1;                   // 16-byte slots per position (odd)
  static constexpr int IMG = SPAN * SLOTS * 16;           // bytes
  static constexpr int WCH = NQ * OCT * 1024;             // bytes of one packed weight chunk
  static constexpr int BUF = WCH + IMG;
  static constexpr int NIT = SPAN * OCT;                  // (position, octet) staging items
  static constexpr int IPT = (NIT + 255) / 256;           // items per thread
  static constexpr int WDMA = NQ * OCT;                   // 1 KiB DMA rows per weight chunk
  static_assert(CK % 16 == 0 && (SLOTS & 1), "k-step = 16 channels; odd slot pitch");
};

#ifndef STGCN_CB1_CK  // chunk channels of the NQ = 1 (spatial / projection) GEMMs
#define STGCN_CB1_CK 16
#endif
#ifndef STGCN_CB1_MINB  // ... and their minimum resident workgroups per CU
#define STGCN_CB1_MINB 2
#endif

// IB: the input is stored in bf16 (p.in_bf16; the NQ = 1 GEMM over a bf16 dZ,
// capi.hip dz_bf16): loaded as zero-extended shorts, packed without conversion
template <int NQ, int CK, int V, int SIN, bool IB = false>
__global__ __launch_bounds__(256, NQ == 1 ? STGCN_CB1_MINB : 2) void k_conv_bf16(ConvGemmParams p) {
  using G = ConvBf16Geo<NQ, CK, V, SIN>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = bid % p.n_rtiles;
  bid /= p.n_rtiles;
  const int mt = bid % p.n_mtiles;
  const int n = bid / p.n_mtiles;
  const int r0 = rt * kTileRows, m0 = mt * G::FT;
  const int cstride = p.T_src * V;
  const int g0 = (SIN * m0 + p.off) * V;
  const float *inN = p.in + (int64_t)n * p.in_bstride;
  const int nchunks = (p.C + CK - 1) / CK;
  const char *wblk = reinterpret_cast<const char *>(p.wpk) + (int64_t)rt * nchunks * G::WCH;
  const int mi = wave & 1, nj0 = (wave >> 1) * 4;

  // per-lane byte offsets of the A fragment and the 4 B fragments (tap 0, octet h)
  const int ao = (hi * 64 + mi * 32 + lo) * 16;
  int bo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = (nj0 + j) * 32 + lo;
    const int mf = col / V;
    const int cp = col < G::NCOLS ? SIN * mf * V + (col - mf * V) : 0;
    bo[j] = (cp * G::SLOTS + hi) * 16;
  }
  // staging items of this thread: (octet o, window position pp); byte offset of
  // channel 8o, position g0 + pp relative to the chunk's first channel
  unsigned voff[G::IPT];
  int loff[G::IPT];
#pragma unroll
  for (int k = 0; k < G::IPT; ++k) {
    const int e = k * 256 + tid;
    const int o = e / G::SPAN, pp = e - o * G::SPAN;
    const int g = g0 + pp;
    const bool ok = e < G::NIT && g >= 0 && g < cstride;
    voff[k] = ok ? (unsigned)(o * 8 * cstride + g) * 4u : kOOB;
    loff[k] = e < G::NIT ? (pp * G::SLOTS + o) * 16 : -1;
  }
  const __amdgpu_buffer_rsrc_t rs_w =
      make_rsrc(reinterpret_cast<const float *>(wblk), (int64_t)nchunks * G::WCH / 4);
  float st[G::IPT][8];
  auto load_img = [&](int chunk) {
    if constexpr (IB) {
      const __bf16 *inb = reinterpret_cast<const __bf16 *>(p.in) + (int64_t)n * p.in_bstride +
                          (int64_t)chunk * CK * cstride;
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(
          reinterpret_cast<const float *>(inb), ((int64_t)(p.C - chunk * CK) * cstride + 1) / 2);
#pragma unroll
      for (int k = 0; k < G::IPT; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          st[k][j] = __builtin_bit_cast(
              float, (unsigned)__builtin_amdgcn_raw_buffer_load_b16(
                         rs, voff[k] == kOOB ? (int)kOOB : (int)((voff[k] >> 1) + j * cstride * 2),
                         0, 0));
    } else {
      const __amdgpu_buffer_rsrc_t rs =
          make_rsrc(inN + (int64_t)chunk * CK * cstride, (int64_t)(p.C - chunk * CK) * cstride);
#pragma unroll
      for (int k = 0; k < G::IPT; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) st[k][j] = ld_f32(rs, voff[k] + (unsigned)(j * cstride * 4));
    }
  };
  auto dma_w = [&](int chunk, char *dst) {
    for (int d = wave; d < G::WDMA; d += 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w, dst + d * 1024, 16,
                                               (unsigned)(chunk * G::WCH + d * 1024 + lane * 16),
                                               0, 0, 0);
  };
  auto write_img = [&](char *dst) {
#pragma unroll
    for (int k = 0; k < G::IPT; ++k)
      if (loff[k] >= 0) {
        uint4 v;
        if constexpr (IB) {  // already bf16 (zero-extended shorts)
          const auto u = [&](int j) { return __builtin_bit_cast(unsigned, st[k][j]); };
          v.x = u(0) | (u(1) << 16);
          v.y = u(2) | (u(3) << 16);
          v.z = u(4) | (u(5) << 16);
          v.w = u(6) | (u(7) << 16);
        } else {
          v.x = pk_bf16(st[k][0], st[k][1]);
          v.y = pk_bf16(st[k][2], st[k][3]);
          v.z = pk_bf16(st[k][4], st[k][5]);
          v.w = pk_bf16(st[k][6], st[k][7]);
        }
        *reinterpret_cast<uint4 *>(dst + loff[k]) = v;
      }
  };

  floatx16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  dma_w(0, lds);
  load_img(0);
  write_img(lds + G::WCH);
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    __syncthreads();  // chunk's weights (DMA) and window (all waves) are in LDS
    char *cur = lds + (chunk & 1) * G::BUF;
    char *nxt = lds + ((chunk + 1) & 1) * G::BUF;
    const bool more = chunk + 1 < nchunks;
    if (more) {
      dma_w(chunk + 1, nxt);
      load_img(chunk + 1);
    }
    const char *wa = cur + ao;
    const char *ib = cur + G::WCH;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int o2 = 0; o2 < G::OCT / 2; ++o2) {
        const bf16x8 a = *reinterpret_cast<const bf16x8 *>(wa + (q * G::OCT + 2 * o2) * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x8 b = *reinterpret_cast<const bf16x8 *>(
              ib + bo[j] + (q * V * G::SLOTS + 2 * o2) * 16);
          acc[j] = mfma_bf16(a, b, acc[j]);
        }
      }
    if (more) write_img(nxt + G::WCH);
  }
  __syncthreads();  // every wave done with the buffers (the epilogue reuses LDS)
  conv_tile_epilogue<V, G::NCOLS, NQ == 1>(p, acc, n, r0, m0, smem);
}

// Packs w[r*w_sr + c*w_sc + q*w_sq] as bf16 into
// wpk[rt][chunk][q][octet][64 rows][8] (zero padded rows and channels).
__global__ void k_pack_conv_w_bf16(const float *w, __bf16 *wpk, int R, int C, int NQ, int CK,
                                   int nch, int64_t w_sr, int64_t w_sc, int64_t w_sq,
                                   int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int jj = (int)(idx & 7);
  int64_t t = idx >> 3;
  const int rl = (int)(t & 63);
  t >>= 6;
  const int oct = CK / 8;
  const int o = (int)(t % oct);
  t /= oct;
  const int q = (int)(t % NQ);
  t /= NQ;
  const int ch = (int)(t % nch);
  const int rt = (int)(t / nch);
  const int r = rt * 64 + rl, c = ch * CK + o * 8 + jj;
  float v = 0.f;
  if (r < R && c < C) v = w[(int64_t)r * w_sr + (int64_t)c * w_sc + (int64_t)q * w_sq];
  wpk[idx] = (__bf16)v;
}

static int conv_bf16_ck(int NQ) { return NQ == 1 ? STGCN_CB1_CK : 16; }

bool conv_bf16_supported(const ConvGemmParams &p) {
  // a reduction over fewer than 16 channels (the first block's C_in = 3: the
  // spatial GEMM over K*3 channels, the 1x1 projection) stays on the fp32
  // path: a bf16 k-step is 16 channels (mostly padding there), and rounding
  // the smooth joint-averaged G of a 3-channel input costs the most precision
  if (p.C < 16) return false;
  if (p.V != 18 && p.V != 25 && p.V != 50) return false;
  if (p.FT != kTileCols / p.V) return false;
  if (p.s_in == 2) return p.NQ == 9 || p.NQ == 1;
  return p.s_in == 1 && (p.NQ == 1 || p.NQ == 4 || p.NQ == 5 || p.NQ == 9);
}

size_t conv_bf16_lds_bytes(const ConvGemmParams &p) {
  const int CK = conv_bf16_ck(p.NQ);
  const int span = (p.s_in * (p.FT - 1) + p.NQ) * p.V;
  const size_t buf = (size_t)p.NQ * (CK / 8) * 1024 + (size_t)span * (CK / 8 + 1) * 16;
  return std::max(2 * buf, (size_t)2048);
}

template <int NQ, int V, int SIN>
static bool launch_cb_if(const ConvGemmParams &p, int nblk, size_t lds, hipStream_t s) {
  if (p.V != V || p.s_in != SIN) return false;
  constexpr int CK = NQ == 1 ? STGCN_CB1_CK : 16;
  if constexpr (NQ == 1 && SIN == 1) {
    if (p.in_bf16) {
      hipLaunchKernelGGL((k_conv_bf16<NQ, CK, V, SIN, true>), dim3(nblk), dim3(256), lds, s, p);
      return true;
    }
  }
  if (p.in_bf16) return false;
  hipLaunchKernelGGL((k_conv_bf16<NQ, CK, V, SIN>), dim3(nblk), dim3(256), lds, s, p);
  return true;
}

template <int NQ, int SIN>
static bool launch_cb_v(const ConvGemmParams &p, int nblk, size_t lds, hipStream_t s) {
  return launch_cb_if<NQ, 18, SIN>(p, nblk, lds, s) || launch_cb_if<NQ, 25, SIN>(p, nblk, lds, s) ||
         launch_cb_if<NQ, 50, SIN>(p, nblk, lds, s);
}

hipError_t launch_conv_bf16(const ConvGemmParams &p, hipStream_t s) {
  // (bf16 input: the NQ = 1 stride-1 GEMM only; no bf16 output here)
  if (!conv_bf16_supported(p) || !p.wpk || p.out_bf16 ||
      (p.in_bf16 && (p.NQ != 1 || p.s_in != 1)))
    return hipErrorInvalidValue;
  const int CK = conv_bf16_ck(p.NQ);
  const int nch = (p.C + CK - 1) / CK;
  {
    const int64_t total = (int64_t)p.n_rtiles * nch * CK * p.NQ * 64;
    hipLaunchKernelGGL(k_pack_conv_w_bf16, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       s, p.w, reinterpret_cast<__bf16 *>(p.wpk), p.R, p.C, p.NQ, CK, nch, p.w_sr,
                       p.w_sc, p.w_sq, total);
  }
  const int nblk = p.N * p.n_mtiles * p.n_rtiles;
  const size_t lds = conv_bf16_lds_bytes(p);
  bool done = false;
  if (p.s_in == 2) {
    done = p.NQ == 9 ? launch_cb_v<9, 2>(p, nblk, lds, s) : launch_cb_v<1, 2>(p, nblk, lds, s);
  } else {
    switch (p.NQ) {
      case 1: done = launch_cb_v<1, 1>(p, nblk, lds, s); break;
      case 4: done = launch_cb_v<4, 1>(p, nblk, lds, s); break;
      case 5: done = launch_cb_v<5, 1>(p, nblk, lds, s); break;
      case 9: done = launch_cb_v<9, 1>(p, nblk, lds, s); break;
    }
  }
  return done ? hipGetLastError() : hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------
// k_wgrad_bf16: the WgradParams weight gradient (internal.h) on bf16 MFMA,
//   slab[split][r][c*NQ + q] = sum_{items of split} sum_{m,v} P[n,r,m,v] Q[n,c,SIN*m+q+off,v]
// NQ = 9 (temporal taps) or 1 (spatial W, residual projection). Output tile
// 64 rows x CB channels x NQ taps; waves = (row half) x (32-channel block) x
// (tap group: taps 0-4 / 5-8 for NQ = 9). Work item = (clip n, FT frames of P);
// the split-K over items is S-way (grid = S x tiles, a split's tiles adjacent),
// each split a contiguous run of items
// The reduction index is the (frame, joint) position with the joint axis
// padded to Vp = round4(V) (P's pad positions are zero, so Q's are don't-care).
// k-step s (16 positions): lane half h takes the position 4-groups 2s, 2s+1 of
// frame half h (frames h*FT/2 ..): eight consecutive positions of P (one
// ds_read_b128) and, per tap, two 4-position runs of Q at frame SIN*m + q
// (two ds_read_b64; row pitches = 4 mod 8 elements: conflict-free).
// Staging: thread t owns position group (t mod PG) of rows t/PG, t/PG + RS, ...
// (PG groups per row, RS = NTH / PG rows per pass), fp32 dword loads through
// a buffer resource (kOOB -> 0 outside the tensor, the halo and the row tail),
// converted and written as 8-byte pieces; double-buffered, one barrier per item.
// ---------------------------------------------------------------------------
template <int NQ, int V, int SIN, int FT, int CB>
struct WgBf16Geo {
  static constexpr int Vp = (V + 3) & ~3;
  static constexpr int G4 = Vp / 4;
  static constexpr int KP = FT * Vp;  // P positions per item
  static constexpr int KSTEPS = KP / 16;
  static constexpr int HF = FT / 2;
  static constexpr int PPITCH = KP + 8;  // elements; PPITCH/8 odd: ds_read_b128 conflict-free
  static constexpr int QF = SIN * (FT - 1) + NQ;  // Q frames per item
  static constexpr int QP0 = QF * Vp;
  static constexpr int QPITCH = QP0 % 8 == 0 ? QP0 + 4 : QP0;  // = 4 mod 8 (b64 conflict-free)
  // tap groups: NQ = 9 -> 2 groups (taps 0-4, 5-8) at CB = 64, 4 groups
  // (0-2, 3-4, 5-6, 7-8) at CB = 32: 8 waves either way
  static constexpr int TG = NQ == 9 ? (CB == 64 ? 2 : 4) : 1;
  static constexpr int NTMAX = NQ == 9 ? (TG == 2 ? 5 : 3) : 1;
  static constexpr int NW = 2 * (CB / 32) * TG;
  static constexpr int NTH = NW * 64;
  static constexpr int PBYTES = (64 * PPITCH * 2 + 15) / 16 * 16;
  static constexpr int QBYTES = (CB * QPITCH * 2 + 15) / 16 * 16;
  static constexpr int BUF = PBYTES + QBYTES;
  // staging: P: PGR = FT*G4 groups per row, RSP rows per pass, NPP passes
  static constexpr int PGR = FT * G4;
  static constexpr int RSP = NTH / PGR;
  static constexpr int NPP = (64 + RSP - 1) / RSP;
  static constexpr int QGR = QF * G4;
  static constexpr int RSQ = NTH / QGR;
  static constexpr int NPQ = (CB + RSQ - 1) / RSQ;
  static constexpr int NPASS = NPP + NPQ;
  static constexpr int NPART = KSTEPS >= 4 ? 4 : 2;  // staging parts per item
  static constexpr int PPART = (NPASS + NPART - 1) / NPART;
  static_assert(KP % 16 == 0 && FT % 2 == 0 && PPITCH % 16 == 8, "k-step geometry");
  static_assert(RSP >= 1 && RSQ >= 1, "a row of position groups fits the workgroup");
};

// BI: P and Q are stored in bf16 (p.p_bf16 == p.q_bf16 == 1; a template switch so
// the staging stays branch-free)
template <int NQ, int V, int SIN, int FT, int CB, bool BI = false>
__global__ __launch_bounds__((WgBf16Geo<NQ, V, SIN, FT, CB>::NTH), 1) void k_wgrad_bf16(WgradParams p) {
  using G = WgBf16Geo<NQ, V, SIN, FT, CB>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  // the tiles of one split are adjacent in the XCD-remapped grid (they read the
  // same items: P rows shared by the column tiles, Q rows by the row tiles, in
  // one L2), and a split takes a CONTIGUOUS run of items (consecutive frame
  // tiles of a clip: the next item's Q halo is mostly this item's frames, L2-hot)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = p.n_rtiles * p.n_jtiles;
  const int tile = bid % ntiles, split = bid / ntiles;
  const int jt = tile % p.n_jtiles;
  const int rt = tile / p.n_jtiles;
  const int r0 = rt * 64, c0 = jt * CB;
  const int mi = wave & 1;
  const int cj = (wave >> 1) % (CB / 32);
  const int tq = wave / (2 * (CB / 32));
  // first tap and tap count of this wave's group
  const int q0 = G::TG == 2 ? 5 * tq : (G::TG == 4 ? (tq ? 1 + 2 * tq : 0) : 0);
  const int nitems = p.N * p.n_mtiles;
  const int per = (nitems + p.S - 1) / p.S;
  const int it0 = min(nitems, split * per), it1 = min(nitems, it0 + per);

  // lane bases (elements) of the A (P) and B (Q) fragments
  const int pa = (mi * 32 + lo) * G::PPITCH + hi * G::HF * G::Vp;
  const int qb = (cj * 32 + lo) * G::QPITCH + hi * SIN * G::HF * G::Vp + q0 * G::Vp;

  // staging geometry of this thread
  const int pg = tid % G::PGR, prow = tid / G::PGR;  // prow >= RSP: idle in P staging
  const int pf = pg / G::G4, pv = (pg % G::G4) * 4;
  const int qg = tid % G::QGR, qrow = tid / G::QGR;
  const int qf = qg / G::G4, qv = (qg % G::G4) * 4;
  const int MV = p.M * V, TV = p.T_src * V;
  // Staging passes: pass k < NPP loads 4 joints of P row prow + k*RSP, pass
  // NPP + k 4 joints of Q row qrow + k*RSQ. An item's passes are issued in
  // NPART parts, each loaded under one NPART-th of the previous item's k-steps
  // and written right after them (fewer staging registers).
  struct ItemRef {
    __amdgpu_buffer_rsrc_t rp, rq;
    bool fok, tok;
    int pbase, qbase;  // element offsets of (row 0 of the tile, frame m0 / t0)
  };
  auto item_ref = [&](int item) {
    ItemRef ir;
    const int n = item / p.n_mtiles, m0 = (item - n * p.n_mtiles) * FT;
    // (p_bf16 / q_bf16: the operand is stored in bf16; resources over its bytes)
    ir.rp = BI ? make_rsrc(reinterpret_cast<const float *>(
                                     reinterpret_cast<const __bf16 *>(p.P) + (int64_t)n * p.p_bstride),
                                 (p.p_bstride + 1) / 2)
                     : make_rsrc(p.P + (int64_t)n * p.p_bstride, p.p_bstride);
    ir.rq = BI ? make_rsrc(reinterpret_cast<const float *>(
                                     reinterpret_cast<const __bf16 *>(p.Q) + (int64_t)n * p.q_bstride),
                                 (p.q_bstride + 1) / 2)
                     : make_rsrc(p.Q + (int64_t)n * p.q_bstride, p.q_bstride);
    ir.fok = prow < G::RSP && m0 + pf < p.M;
    const int t = SIN * m0 + p.off + qf;
    ir.tok = qrow < G::RSQ && t >= 0 && t < p.T_src;
    ir.pbase = (m0 + pf) * V + pv;
    ir.qbase = t * V + qv;
    return ir;
  };
  float st[G::PPART][4];
  auto load_part = [&](const ItemRef &ir, auto part_c) {
    constexpr int PART = decltype(part_c)::value;
#pragma unroll
    for (int i = 0; i < G::PPART; ++i) {
      const int k = PART * G::PPART + i;
      if (k < G::NPP) {
        const int r = r0 + prow + k * G::RSP;
        const bool ok = ir.fok && prow + k * G::RSP < 64 && r < p.R;
        const unsigned base = ok ? (unsigned)(r * MV + ir.pbase) * (BI ? 2u : 4u) : kOOB;
        if constexpr (BI) {  // packed pairs in st[i][0..1]; pad joints (>= V) zeroed
          unsigned x, y;
          ld_b16x4<V % 2 == 1>(ir.rp, base, x, y);
          if (pv + 1 >= V) x &= 0xffffu;
          if (pv + 2 >= V) y = 0u;
          else if (pv + 3 >= V) y &= 0xffffu;
          st[i][0] = __builtin_bit_cast(float, x);
          st[i][1] = __builtin_bit_cast(float, y);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            st[i][j] = (pv + j < V) ? ld_f32(ir.rp, base + 4u * j) : 0.f;  // pad joints: 0
        }
      } else if (k < G::NPP + G::NPQ) {
        const int kq = k - G::NPP;
        const int c = c0 + qrow + kq * G::RSQ;
        const bool ok = ir.tok && qrow + kq * G::RSQ < CB && c < p.C;
        const unsigned base = ok ? (unsigned)(c * TV + ir.qbase) * (BI ? 2u : 4u) : kOOB;
        if constexpr (BI) {
          unsigned x, y;
          ld_b16x4<V % 2 == 1>(ir.rq, base, x, y);
          st[i][0] = __builtin_bit_cast(float, x);
          st[i][1] = __builtin_bit_cast(float, y);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) st[i][j] = ld_f32(ir.rq, base + 4u * j);
        }
      }
    }
  };
  auto write_part = [&](char *buf, auto part_c) {
    constexpr int PART = decltype(part_c)::value;
#pragma unroll
    for (int i = 0; i < G::PPART; ++i) {
      const int k = PART * G::PPART + i;
      uint2 v;
      if constexpr (BI) {  // already packed bf16 pairs
        v.x = __builtin_bit_cast(unsigned, st[i][0]);
        v.y = __builtin_bit_cast(unsigned, st[i][1]);
      } else {
        v.x = pk_bf16(st[i][0], st[i][1]);
        v.y = pk_bf16(st[i][2], st[i][3]);
      }
      if (k < G::NPP) {
        if (prow < G::RSP && prow + k * G::RSP < 64)
          *reinterpret_cast<uint2 *>(buf + ((prow + k * G::RSP) * G::PPITCH + pf * G::Vp + pv) * 2) = v;
      } else if (k < G::NPP + G::NPQ) {
        const int kq = k - G::NPP;
        if (qrow < G::RSQ && qrow + kq * G::RSQ < CB)
          *reinterpret_cast<uint2 *>(buf + G::PBYTES +
                                     ((qrow + kq * G::RSQ) * G::QPITCH + qf * G::Vp + qv) * 2) = v;
      }
    }
  };

  constexpr int NTMAX = G::NTMAX;

  // k-loop with the operands of step s+1 read (LDS) under the MFMAs of step s
  auto compute = [&](floatx16 *acc, const char *buf, auto nt_c, auto s0_c, auto s1_c) {
    constexpr int NT = decltype(nt_c)::value;
    constexpr int S0 = decltype(s0_c)::value, S1 = decltype(s1_c)::value;
    const __bf16 *P = reinterpret_cast<const __bf16 *>(buf) + pa;
    const __bf16 *Q = reinterpret_cast<const __bf16 *>(buf + G::PBYTES) + qb;
    bf16x8 a[2], b[2][NT];
    auto ld = [&](int s, int set) {
      a[set] = *reinterpret_cast<const bf16x8 *>(P + 8 * s);
      // position 4-groups 2s, 2s+1 of the frame half: Q frame SIN*m + tap, joint v0
      const int ga = 2 * s, gb = 2 * s + 1;
      const int oa = SIN * (ga / G::G4) * G::Vp + (ga % G::G4) * 4;
      const int ob = SIN * (gb / G::G4) * G::Vp + (gb % G::G4) * 4;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const bf16x4 b0 = *reinterpret_cast<const bf16x4 *>(Q + oa + t * G::Vp);
        const bf16x4 b1 = *reinterpret_cast<const bf16x4 *>(Q + ob + t * G::Vp);
        b[set][t] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    };
    ld(S0, 0);
#pragma unroll
    for (int s = S0; s < S1; ++s) {
      if (s + 1 < S1) ld(s + 1, (s + 1 - S0) & 1);
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = mfma_bf16(a[(s - S0) & 1], b[(s - S0) & 1][t], acc[t]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // one item: part j of the next item's staging is loaded under the j-th
  // slice of this item's k-steps and written after it
  auto item_body = [&](floatx16 *acc, const char *cur, char *nxt, bool more, const ItemRef &nir,
                       auto nt_c) {
    auto part = [&](auto j_c) {
      constexpr int J = decltype(j_c)::value;
      constexpr int S0 = J * G::KSTEPS / G::NPART, S1 = (J + 1) * G::KSTEPS / G::NPART;
      if (more) load_part(nir, j_c);
      compute(acc, cur, nt_c, std::integral_constant<int, S0>{}, std::integral_constant<int, S1>{});
      if (more) write_part(nxt, j_c);
    };
    part(std::integral_constant<int, 0>{});
    part(std::integral_constant<int, 1>{});
    if constexpr (G::NPART == 4) {
      part(std::integral_constant<int, 2>{});
      part(std::integral_constant<int, 3>{});
    }
  };

  // LDS-DMA staging (bf16 P and Q, even V: a frame's joints are whole dwords, so
  // 4-byte LDS-DMA pieces land in the padded frame image without realignment).
  // Dword d of a buffer's P image (Q image) is (row, frame f, joint pair j) of
  // the same layout the register staging writes; its source element offset
  // within the clip minus the item's frame base is fixed per lane and wave
  // round, kept in a register as (f << 26 | offset) (~0: pitch pad, pad joint
  // or row past the tensor -> OOB -> 0). An item's whole staging is in flight
  // under the previous item's k-steps; one vmcnt(0) + barrier per item.
  constexpr bool DMA = BI && NQ == 9 && V % 2 == 0 && !STGCN_AB_WG_REGSTAGE;
  constexpr int PW = G::PPITCH / 2, QW = G::QPITCH / 2, VW = G::Vp / 2;  // dwords
  constexpr int PRN = 64 * PW / 64, QRN = CB * QW / 64;  // wave rounds of 64 dwords
  constexpr int PR = (PRN + G::NW - 1) / G::NW, QR = (QRN + G::NW - 1) / G::NW;
  static_assert(!DMA || (G::PBYTES == 64 * PW * 4 && (CB * QW) % 64 == 0), "whole wave rounds");
  // (offsets must fit 26 bits; block-uniform, else the register staging runs)
  const bool dma_ok = DMA && (int64_t)p.R * MV < (1 << 26) && (int64_t)p.C * TV < (1 << 26);
  unsigned ptab[DMA ? PR : 1], qtab[DMA ? QR : 1];
  if constexpr (DMA) {
#pragma unroll
    for (int i = 0; i < PR; ++i) {
      const int d = (i * G::NW + wave) * 64 + lane;
      const int row = d / PW, w = d - row * PW, f = w / VW, j = w - f * VW;
      const bool ok = i * G::NW + wave < PRN && f < FT && 2 * j < V && r0 + row < p.R;
      ptab[i] = ok ? ((unsigned)f << 26) | (unsigned)((r0 + row) * MV + f * V + 2 * j) : ~0u;
    }
#pragma unroll
    for (int i = 0; i < QR; ++i) {
      const int d = (i * G::NW + wave) * 64 + lane;
      const int c = d / QW, w = d - c * QW, f = w / VW, j = w - f * VW;
      const bool ok = i * G::NW + wave < QRN && f < G::QF && 2 * j < V && c0 + c < p.C;
      qtab[i] = ok ? ((unsigned)f << 26) | (unsigned)((c0 + c) * TV + f * V + 2 * j) : ~0u;
    }
  }
  const unsigned lds_addr = (unsigned)reinterpret_cast<uintptr_t>(lds);
  auto dma_stage = [&](int item, int bufi) __attribute__((always_inline)) {
    const int n = item / p.n_mtiles, m0 = (item - n * p.n_mtiles) * FT;
    const uint64_t sp = reinterpret_cast<uint64_t>(reinterpret_cast<const __bf16 *>(p.P) +
                                                   (int64_t)n * p.p_bstride);
    const uint64_t sq = reinterpret_cast<uint64_t>(reinterpret_cast<const __bf16 *>(p.Q) +
                                                   (int64_t)n * p.q_bstride);
    const int4v rp = uniform4(int4v{(int)(uint32_t)sp, (int)((sp >> 32) & 0xffff),
                               (int)std::min<int64_t>(p.p_bstride * 2, 0x7fffffff), 0x00020000});
    const int4v rq = uniform4(int4v{(int)(uint32_t)sq, (int)((sq >> 32) & 0xffff),
                               (int)std::min<int64_t>(p.q_bstride * 2, 0x7fffffff), 0x00020000});
    const int t0 = SIN * m0 + p.off;
    const unsigned lb =
        (unsigned)__builtin_amdgcn_readfirstlane((int)(lds_addr + (unsigned)(bufi * G::BUF)));
    asm volatile("s_nop 4" ::: "memory");  // descriptor SGPRs -> buffer_load
#pragma unroll
    for (int i = 0; i < PR; ++i)
      if (i * G::NW + wave < PRN) {
        const unsigned e = ptab[i];
        const bool ok = e != ~0u && m0 + (int)(e >> 26) < p.M;
        const unsigned voff = ok ? ((e & 0x3ffffffu) + (unsigned)(m0 * V)) * 2u : kOOB;
        dma_b32(rp, voff, lb + (unsigned)((i * G::NW + wave) * 256));
      }
#pragma unroll
    for (int i = 0; i < QR; ++i)
      if (i * G::NW + wave < QRN) {
        const unsigned e = qtab[i];
        const int t = t0 + (int)(e >> 26);
        const bool ok = e != ~0u && t >= 0 && t < p.T_src;
        const unsigned voff = ok ? (unsigned)((int)(e & 0x3ffffffu) + t0 * V) * 2u : kOOB;
        dma_b32(rq, voff, lb + (unsigned)(G::PBYTES + (i * G::NW + wave) * 256));
      }
  };

  if (!dma_ok && it0 < it1) {
    const ItemRef ir = item_ref(it0);
    load_part(ir, std::integral_constant<int, 0>{});
    write_part(lds, std::integral_constant<int, 0>{});
    load_part(ir, std::integral_constant<int, 1>{});
    write_part(lds, std::integral_constant<int, 1>{});
    if constexpr (G::NPART == 4) {
      load_part(ir, std::integral_constant<int, 2>{});
      write_part(lds, std::integral_constant<int, 2>{});
      load_part(ir, std::integral_constant<int, 3>{});
      write_part(lds, std::integral_constant<int, 3>{});
    }
  }
  // the item loop and the slab store, instantiated per tap count of the wave
  // (a wave-uniform branch outside the loop: the accumulators of the two
  // variants never meet)
  auto run = [&](auto nt_c) {
    constexpr int NT = decltype(nt_c)::value;
    floatx16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    if (dma_ok) {
      if (it0 < it1) dma_stage(it0, 0);
      for (int it = 0, itm = it0; itm < it1; ++it, ++itm) {
        // item it landed (every wave's pieces), and every wave is done reading
        // item it-1's buffer, which item it+1's pieces overwrite
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (itm + 1 < it1) dma_stage(itm + 1, (it + 1) & 1);
        compute(acc, lds + (it & 1) * G::BUF, nt_c, std::integral_constant<int, 0>{},
                std::integral_constant<int, G::KSTEPS>{});
      }
    } else
    for (int it = 0, itm = it0; itm < it1; ++it, ++itm) {
      __syncthreads();
      const char *cur = lds + (it & 1) * G::BUF;
      char *nxt = lds + ((it + 1) & 1) * G::BUF;
      const bool more = itm + 1 < it1;
      const ItemRef nir = item_ref(more ? itm + 1 : itm);
      item_body(acc, cur, nxt, more, nir, nt_c);
    }
    // partial tile -> slab[split][r][c*NQ + q]
    float *slab = p.slab + (int64_t)split * p.R * p.C * NQ;
    const int c = c0 + cj * 32 + lo;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r = r0 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
        if (r < p.R && c < p.C) slab[((int64_t)r * p.C + c) * NQ + q0 + t] = acc[t][i];
      }
  };
  if (tq == 0)  // the first tap group has the most taps
    run(std::integral_constant<int, NTMAX>{});
  else
    run(std::integral_constant<int, (NTMAX > 1 ? NTMAX - 1 : 1)>{});
}

// ---------------------------------------------------------------------------
// k_wgrad_bf16_raw: the stride-1 temporal weight gradient for bf16 P / Q at
// V = 25 (odd: a frame's joints are not whole dwords, so the padded-frame
// images of k_wgrad_bf16 cannot be filled by dword LDS-DMA). Same tiles, items
// (clip, FT = 4 frames), split-K plan and slab as k_wgrad_bf16<9,25,1,4,64>, but
// the reduction index is the item's RAW position k = f V + v (100 positions,
// 7 k-steps of 16; P zero past 100), so an item's rows are contiguous runs in
// HBM that start on even elements whenever the clip's frame counts are even
// (M = T_src even: the host checks) and move by 4-byte LDS-DMA pieces straight
// into the images: P [64][120] and the Q window [64 channels][314] (frames
// m0-4 .. m0+7, zero outside [0, T)). Tap q reads Q at k + 25 q: the B fragment
// (8 consecutive positions) starts on an odd element for odd q, so it is read as
// 5 dwords and realigned with v_alignbit (4 aligned dwords for even q). Whole
// next item in flight under the current one, one vmcnt(0) + barrier per item.
// ---------------------------------------------------------------------------
struct WgRawGeo {
  static constexpr int V = 25, FT = 4, CB = 64, NQ = 9;
  static constexpr int KP = FT * V;                 // 100 positions
  static constexpr int KSTEPS = (KP + 15) / 16;     // 7
  static constexpr int PP = 120;                    // P pitch (elements): PP/8 odd
  static constexpr int QW = (FT + 8) * V;           // 300 window elements
  static constexpr int QPD = 157;                   // Q pitch (dwords, odd) >= (111 + 200 + 3) / 2
  static constexpr int PDW = 64 * PP / 2;           // 3840 dwords
  static constexpr int QDW = CB * QPD;              // 10048 dwords
  static constexpr int PBYTES = PDW * 4, BUF = (PDW + QDW) * 4;
  static constexpr int NW = 8;
  static constexpr int PRN = PDW / 64, QRN = QDW / 64;  // 60, 157 wave rounds
  static constexpr int PR = (PRN + NW - 1) / NW, QR = (QRN + NW - 1) / NW;
  static_assert(PDW % 64 == 0 && QDW % 64 == 0, "whole wave rounds");
  static_assert(2 * BUF <= 160 * 1024, "LDS budget");
};

bool wgrad_raw_ok(const WgradParams &p) {
  return p.NQ == 9 && p.V == 25 && p.s_in == 1 && p.off == -4 && p.FT == 4 && p.p_bf16 &&
         p.q_bf16 && p.M % 2 == 0 && p.T_src % 2 == 0 && (int64_t)p.R * p.M * 25 < (1 << 23) &&
         (int64_t)p.C * p.T_src * 25 < (1 << 23) && p.n_jtiles * 64 >= p.C &&
         !STGCN_AB_WG_REGSTAGE;
}

__global__ __launch_bounds__(512, 1) void k_wgrad_bf16_raw(WgradParams p) {
  using G = WgRawGeo;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = p.n_rtiles * p.n_jtiles;
  const int tile = bid % ntiles, split = bid / ntiles;
  const int jt = tile % p.n_jtiles, rt = tile / p.n_jtiles;
  const int r0 = rt * 64, c0 = jt * G::CB;
  const int mi = wave & 1, cj = (wave >> 1) & 1, tq = wave >> 2;  // taps 0-4 / 5-8
  const int nitems = p.N * p.n_mtiles;
  const int per = (nitems + p.S - 1) / p.S;
  const int it0 = min(nitems, split * per), it1 = min(nitems, it0 + per);
  const int MV = p.M * G::V, TV = p.T_src * G::V;

  // per-lane DMA tables: (frame of the dword's first element << 23) | element
  // offset within the clip (without the item's frame base); ~0: pad / past the tensor
  unsigned ptab[G::PR], qtab[G::QR];
#pragma unroll
  for (int i = 0; i < G::PR; ++i) {
    const int d = (i * G::NW + wave) * 64 + lane;
    const int row = d / (G::PP / 2), e = 2 * (d - row * (G::PP / 2));
    const bool ok = i * G::NW + wave < G::PRN && e < G::KP && r0 + row < p.R;
    ptab[i] = ok ? ((unsigned)(e / G::V) << 23) | (unsigned)((r0 + row) * MV + e) : ~0u;
  }
#pragma unroll
  for (int i = 0; i < G::QR; ++i) {
    const int d = (i * G::NW + wave) * 64 + lane;
    const int c = d / G::QPD, e = 2 * (d - c * G::QPD);
    const bool ok = i * G::NW + wave < G::QRN && e < G::QW && c0 + c < p.C;
    qtab[i] = ok ? ((unsigned)(e / G::V) << 23) | (unsigned)((c0 + c) * TV + e) : ~0u;
  }
  const unsigned lds_addr = (unsigned)reinterpret_cast<uintptr_t>(lds);
  auto stage = [&](int item, int bufi) __attribute__((always_inline)) {
    const int n = item / p.n_mtiles, m0 = (item - n * p.n_mtiles) * G::FT;
    const uint64_t sp = reinterpret_cast<uint64_t>(reinterpret_cast<const __bf16 *>(p.P) +
                                                   (int64_t)n * p.p_bstride);
    const uint64_t sq = reinterpret_cast<uint64_t>(reinterpret_cast<const __bf16 *>(p.Q) +
                                                   (int64_t)n * p.q_bstride);
    const int4v rp = uniform4(int4v{(int)(uint32_t)sp, (int)((sp >> 32) & 0xffff),
                                    (int)std::min<int64_t>(p.p_bstride * 2, 0x7fffffff), 0x00020000});
    const int4v rq = uniform4(int4v{(int)(uint32_t)sq, (int)((sq >> 32) & 0xffff),
                                    (int)std::min<int64_t>(p.q_bstride * 2, 0x7fffffff), 0x00020000});
    const int t0 = m0 - 4;
    const unsigned lb =
        (unsigned)__builtin_amdgcn_readfirstlane((int)(lds_addr + (unsigned)(bufi * G::BUF)));
    asm volatile("s_nop 4" ::: "memory");  // descriptor SGPRs -> buffer_load
#pragma unroll
    for (int i = 0; i < G::PR; ++i)
      if (i * G::NW + wave < G::PRN) {
        const unsigned e = ptab[i];
        const bool ok = e != ~0u && m0 + (int)(e >> 23) < p.M;
        const unsigned voff = ok ? ((e & 0x7fffffu) + (unsigned)(m0 * G::V)) * 2u : kOOB;
        dma_b32(rp, voff, lb + (unsigned)((i * G::NW + wave) * 256));
      }
#pragma unroll
    for (int i = 0; i < G::QR; ++i)
      if (i * G::NW + wave < G::QRN) {
        const unsigned e = qtab[i];
        const int t = t0 + (int)(e >> 23);
        const bool ok = e != ~0u && t >= 0 && t < p.T_src;
        const unsigned voff = ok ? (unsigned)((int)(e & 0x7fffffu) + t0 * G::V) * 2u : kOOB;
        dma_b32(rq, voff, lb + (unsigned)(G::PBYTES + (i * G::NW + wave) * 256));
      }
  };

  auto run = [&](auto q0_c, auto nt_c) {
    constexpr int Q0 = decltype(q0_c)::value, NT = decltype(nt_c)::value;
    floatx16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    const int pa = (mi * 32 + lo) * G::PP + 8 * hi;            // elements
    const int qd = (cj * 32 + lo) * G::QPD;                      // dwords
    auto compute = [&](const char *buf) {
      const __bf16 *P = reinterpret_cast<const __bf16 *>(buf) + pa;
      const unsigned *Qd = reinterpret_cast<const unsigned *>(buf + G::PBYTES) + qd;
      auto ldb = [&](int s, int t) {
        constexpr int dummy = 0;
        (void)dummy;
        const int q = Q0 + t;
        const int e0 = 16 * s + 8 * hi + 25 * q;  // first element of the fragment
        const unsigned *src = Qd + (e0 >> 1);
        unsigned u[5];
#pragma unroll
        for (int j = 0; j < 4; ++j) u[j] = src[j];
        uint4 w;
        if (q & 1) {  // odd start: elements from the high half of dword 0
          u[4] = src[4];
          w.x = __builtin_amdgcn_alignbit(u[1], u[0], 16);
          w.y = __builtin_amdgcn_alignbit(u[2], u[1], 16);
          w.z = __builtin_amdgcn_alignbit(u[3], u[2], 16);
          w.w = __builtin_amdgcn_alignbit(u[4], u[3], 16);
        } else {
          w = make_uint4(u[0], u[1], u[2], u[3]);
        }
        return __builtin_bit_cast(bf16x8, w);
      };
      bf16x8 a[2], b[2][NT];
      auto ld = [&](int s, int set) {
        a[set] = *reinterpret_cast<const bf16x8 *>(P + 16 * s);
#pragma unroll
        for (int t = 0; t < NT; ++t) b[set][t] = ldb(s, t);
      };
      ld(0, 0);
#pragma unroll
      for (int s = 0; s < G::KSTEPS; ++s) {
        if (s + 1 < G::KSTEPS) ld(s + 1, (s + 1) & 1);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma_bf16(a[s & 1], b[s & 1][t], acc[t]);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (it0 < it1) stage(it0, 0);
    for (int it = 0, itm = it0; itm < it1; ++it, ++itm) {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (itm + 1 < it1) stage(itm + 1, (it + 1) & 1);
      compute(lds + (it & 1) * G::BUF);
    }
    float *slab = p.slab + (int64_t)split * p.R * p.C * G::NQ;
    const int c = c0 + cj * 32 + lo;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r = r0 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
        if (r < p.R && c < p.C) slab[((int64_t)r * p.C + c) * G::NQ + Q0 + t] = acc[t][i];
      }
  };
  if (tq == 0)
    run(std::integral_constant<int, 0>{}, std::integral_constant<int, 5>{});
  else
    run(std::integral_constant<int, 5>{}, std::integral_constant<int, 4>{});
}

// ---------------------------------------------------------------------------
// k_wgrad_gemm_bf16: the NQ = 1, stride-1 weight gradient (the spatial
// dW' = dZ G^T) as a plain split-K GEMM over the contiguous (t, v) positions of
// each clip row: slab[split][r][c] = sum_{items} sum_{l in chunk} P[n][r][l] Q[n][c][l].
// A bandwidth-bound GEMM (every P row is re-read by C/TC column tiles, every Q
// row by R/TR row tiles): big tiles (TR x TC = 128 x 256, 8 waves of 64 x 64)
// for reuse, operands staged in fp32 by LDS-DMA straight from HBM (no staging
// registers, coalesced rows; 16-byte pieces when rows are 16-byte aligned),
// rounded to bf16 when the MFMA fragments are read (2 x ds_read_b128 + 4
// v_cvt_pk_bf16_f32 per fragment). Item = (clip, KC = 32 positions);
// double-buffered; the WGs of one split are adjacent in the (XCD-remapped)
// grid so they share the split's chunks in L2.
// ---------------------------------------------------------------------------
template <int TR, int TC>
struct WgGemmGeo {
  static constexpr int KC = 32, PITCH = KC + 4;  // floats (PITCH/4 odd: b128 conflict-free)
  static constexpr int PSZ = TR * PITCH, QSZ = TC * PITCH, BUF = PSZ + QSZ;  // floats
  static constexpr int NWR = TR / 64, NWC = TC / 64, NW = NWR * NWC;
  static constexpr int NTH = NW * 64;
};

template <int TR, int TC, bool X4>
__global__ __launch_bounds__((WgGemmGeo<TR, TC>::NTH), 1) void k_wgrad_gemm_bf16(WgradParams p) {
  using G = WgGemmGeo<TR, TC>;
  constexpr int GF = X4 ? 4 : 1;                              // floats per lane per DMA
  constexpr int ROUNDS = (G::BUF / GF + G::NTH - 1) / G::NTH;  // DMA rounds per wave
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = p.n_rtiles * p.n_jtiles;
  const int tile = bid % ntiles;
  const int split = bid / ntiles;
  const int ct = tile % p.n_jtiles, rt = tile / p.n_jtiles;
  const int L = p.M * p.V;
  const int r0 = rt * TR, c0 = ct * TC;
  const int prow_lim = min(TR, p.R - r0), qrow_lim = min(TC, p.C - c0);
  const int total = p.N * p.n_mtiles;
  const int per = (total + p.S - 1) / p.S;
  const int it0 = split * per, it1 = min(total, it0 + per);

  // DMA round i of this wave fills image floats [((i*NW + wave)*64 + lane)*GF, +GF);
  // the image is P rows [0, TR) then Q rows, PITCH floats each
  int goff[ROUNDS], gcol[ROUNDS];
#pragma unroll
  for (int i = 0; i < ROUNDS; ++i) {
    const int pos = ((i * G::NW + wave) * 64 + lane) * GF;
    const int row = pos / G::PITCH, col = pos - row * G::PITCH;
    const bool isq = row >= TR;
    const int rr = isq ? row - TR : row;
    gcol[i] = col;
    goff[i] = (pos < G::BUF && col < G::KC && rr < (isq ? qrow_lim : prow_lim)) ? rr * L + col : -1;
  }
  auto stage = [&](int it, float *buf) {
    const int n = it / p.n_mtiles, kc = it - n * p.n_mtiles;
    const int l0 = kc * G::KC, lrem = L - l0;
    const __amdgpu_buffer_rsrc_t rs_p = make_rsrc(
        p.P + (int64_t)n * p.p_bstride + (int64_t)r0 * L + l0, (int64_t)prow_lim * L - l0);
    const __amdgpu_buffer_rsrc_t rs_q = make_rsrc(
        p.Q + (int64_t)n * p.q_bstride + (int64_t)c0 * L + l0, (int64_t)qrow_lim * L - l0);
#pragma unroll
    for (int i = 0; i < ROUNDS; ++i) {
      const int base = (i * G::NW + wave) * 64 * GF;  // wave-uniform
      if (base < G::BUF) {
        const bool isq = base >= G::PSZ;  // rounds never straddle P and Q (PSZ % (64*GF) == 0)
        const bool ok = goff[i] >= 0 && gcol[i] < lrem;
        const unsigned voff = ok ? (unsigned)goff[i] * 4u : kOOB;
        if constexpr (X4)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(isq ? rs_q : rs_p, buf + base, 16, voff, 0, 0, 0);
        else
          blds_f32(isq ? rs_q : rs_p, voff, buf + base);
      }
    }
  };
  const int wr = wave / G::NWC, wc = wave % G::NWC;  // this wave's 64 x 64 sub-tile
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // 8 consecutive fp32 -> bf16x8, as two 16-byte LDS reads (fragment rows are
  // 16-byte aligned; element-wise reads compiled to b96 + b32 pieces)
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  auto frag = [&](const float *src) {
    const f32x4v *v = reinterpret_cast<const f32x4v *>(__builtin_assume_aligned(src, 16));
    const f32x4v l4 = v[0], h4 = v[1];
    return bf16x8{(__bf16)l4.x, (__bf16)l4.y, (__bf16)l4.z, (__bf16)l4.w,
                  (__bf16)h4.x, (__bf16)h4.y, (__bf16)h4.z, (__bf16)h4.w};
  };
  float *buf0 = smem, *buf1 = smem + G::BUF;
  if (it0 < it1) stage(it0, buf0);
  __syncthreads();
  for (int it = it0; it < it1; ++it) {
    const bool odd = (it - it0) & 1;
    const float *cur = odd ? buf1 : buf0;
    if (it + 1 < it1) stage(it + 1, odd ? buf0 : buf1);
    const float *pa = cur + (wr * 64 + lo) * G::PITCH + 8 * hi;
    const float *qb = cur + G::PSZ + (wc * 64 + lo) * G::PITCH + 8 * hi;
#pragma unroll
    for (int s = 0; s < G::KC / 16; ++s) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = frag(pa + i * 32 * G::PITCH + 16 * s);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = frag(qb + j * 32 * G::PITCH + 16 * s);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf16(a[i], b[j], acc[i][j]);
    }
    __syncthreads();  // retires this wave's LDS-DMA and publishes the next chunk
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

// Tile plans (FT, CB) per (NQ, V, SIN): double-buffered images within 160 KiB.
struct WgBf16Plan {
  int FT, CB;
};

static bool wgrad_bf16_plan(const WgradParams &w, WgBf16Plan &pl) {
  if (w.V != 18 && w.V != 25 && w.V != 50) return false;
  if (w.s_in != 1 && w.s_in != 2) return false;
  if (w.NQ == 9) {
    if (w.off != -4) return false;
    pl.FT = w.V == 18 ? 8 : 4;
    pl.CB = w.V == 50 ? 32 : 64;
  } else if (w.NQ == 1) {
    if (w.off != 0) return false;
    pl.FT = 4;
    pl.CB = 64;
  } else {
    return false;
  }
  return true;
}

bool plan_wgrad_bf16(WgradParams &w) {
  if (w.NQ == 1 && w.s_in == 1 && w.off == 0 && w.M == w.T_src) {
    // plain split-K GEMM over contiguous positions (k_wgrad_gemm_bf16); FT = 0
    // marks the plan, CT = rows per tile (128 | 64), columns per tile 256
    w.FT = 0;
    w.CT = w.R > 64 ? 128 : 64;
    w.n_mtiles = (w.M * w.V + 31) / 32;
    w.n_rtiles = (w.R + w.CT - 1) / w.CT;
    w.n_jtiles = (w.C + 255) / 256;
    const int tiles = w.n_rtiles * w.n_jtiles;
    w.S = std::max(1, std::min((256 + tiles - 1) / tiles, w.N * w.n_mtiles));
    w.bf16 = 1;
    return true;
  }
  WgBf16Plan pl;
  if (!wgrad_bf16_plan(w, pl)) return false;
  w.FT = pl.FT;
  w.n_mtiles = (w.M + pl.FT - 1) / pl.FT;
  w.n_rtiles = (w.R + 63) / 64;
  w.n_jtiles = (w.C + pl.CB - 1) / pl.CB;
  const int tiles = w.n_rtiles * w.n_jtiles;
  const int target = w.NQ == 9 ? 256 : 512;
  w.S = std::max(1, std::min((target + tiles - 1) / tiles, w.N * w.n_mtiles));
  w.bf16 = 1;
  return true;
}

template <int NQ, int V, int SIN, int FT, int CB>
static bool launch_wb_if(const WgradParams &p, hipStream_t s) {
  if (p.V != V || p.s_in != SIN || p.FT != FT) return false;
  using G = WgBf16Geo<NQ, V, SIN, FT, CB>;
  const int nblk = p.n_rtiles * p.n_jtiles * p.S;
  if constexpr (NQ == 9) {  // (bf16 P and Q: the temporal weight gradient only)
    if constexpr (V == 25 && SIN == 1) {
      if (wgrad_raw_ok(p)) {  // raw positions by LDS-DMA (odd V)
        hipLaunchKernelGGL(k_wgrad_bf16_raw, dim3(nblk), dim3(512), 2 * WgRawGeo::BUF, s, p);
        return true;
      }
    }
    if (p.p_bf16 && p.q_bf16) {
      hipLaunchKernelGGL((k_wgrad_bf16<NQ, V, SIN, FT, CB, true>), dim3(nblk), dim3(G::NTH),
                         2 * G::BUF, s, p);
      return true;
    }
  }
  if (p.p_bf16 || p.q_bf16) return false;
  hipLaunchKernelGGL((k_wgrad_bf16<NQ, V, SIN, FT, CB>), dim3(nblk), dim3(G::NTH), 2 * G::BUF, s,
                     p);
  return true;
}

template <int TR, bool X4>
static void launch_wgg(const WgradParams &p, int nblk, hipStream_t s) {
  using G = WgGemmGeo<TR, 256>;
  hipLaunchKernelGGL((k_wgrad_gemm_bf16<TR, 256, X4>), dim3(nblk), dim3(G::NTH),
                     2 * G::BUF * sizeof(float), s, p);
}

hipError_t launch_wgrad_bf16(const WgradParams &p, hipStream_t s) {
  if (!p.bf16) return hipErrorInvalidValue;
  if (p.NQ == 1 && p.FT == 0) {
    const int nblk = p.n_rtiles * p.n_jtiles * p.S;
    const int64_t L = (int64_t)p.M * p.V;
    const bool x4 = L % 4 == 0 && p.p_bstride % 4 == 0 && p.q_bstride % 4 == 0 &&
                    ((uintptr_t)p.P & 15) == 0 && ((uintptr_t)p.Q & 15) == 0;
    if (p.CT == 128) {
      if (x4) launch_wgg<128, true>(p, nblk, s); else launch_wgg<128, false>(p, nblk, s);
    } else {
      if (x4) launch_wgg<64, true>(p, nblk, s); else launch_wgg<64, false>(p, nblk, s);
    }
    return hipGetLastError();
  }
  bool done = false;
  if (p.NQ == 9) {
    done = launch_wb_if<9, 18, 1, 8, 64>(p, s) || launch_wb_if<9, 18, 2, 8, 64>(p, s) ||
           launch_wb_if<9, 25, 1, 4, 64>(p, s) || launch_wb_if<9, 25, 2, 4, 64>(p, s) ||
           launch_wb_if<9, 50, 1, 4, 32>(p, s) || launch_wb_if<9, 50, 2, 4, 32>(p, s);
  } else if (p.NQ == 1) {
    done = launch_wb_if<1, 18, 1, 4, 64>(p, s) || launch_wb_if<1, 18, 2, 4, 64>(p, s) ||
           launch_wb_if<1, 25, 1, 4, 64>(p, s) || launch_wb_if<1, 25, 2, 4, 64>(p, s) ||
           launch_wb_if<1, 50, 1, 4, 64>(p, s) || launch_wb_if<1, 50, 2, 4, 64>(p, s);
  }
  return done ? hipGetLastError() : hipErrorInvalidValue;
}

}  // namespace stgcn

// Fused SpatialConv backward of the bf16 path (STGCN_F_BF16) — gfx950 only.
//
// k_sp_bwd_fused<V, K>: the backward of the spatial graph convolution in the
// form (1) of capi.hip, from dZ (the gradient at the SpatialConv output,
// st_graphconv.py:139-152) to dxhat, dA and the BN1 backward sums, in ONE
// kernel, so the K*C_in-channel H = W'^T dZ never reaches HBM (the unfused
// path writes H with a channel GEMM and reads it back in k_spatial_bwd5/6):
//   H_k[ci][t][v]  = sum_r W_k[r][ci] dZ[r][t][v]           (channel GEMM, MFMA)
//   dxhat[ci][t][w] = sum_k sum_v H_k[ci][t][v] A_k[v][w]   (joint contraction)
//   dA_k[v][w]    += sum_{ci,t} H_k[ci][t][v] f(BN1(x))[ci][t][w]
//   sd[ci] += sum dx, sdn[ci] += sum dx * xhat (BN1 backward), dx = dxhat
//   (f = ReLU in the residual block, st_graphconv.py:72-74: dx masked where
//   BN1(x) <= 0)
// Persistent grid, one 8-wave workgroup per CU; work item = (clip n, frame tile
// of FT frames, 32 input channels). Wave w owns frame f = w / NVT and the
// 32-joint tile vt = w % NVT of that frame (NVT = 1 for V = 25, 2 for V = 50)
// and computes its H tiles in BOTH orientations from the same fragments:
//   T_k = H_k^T  (rows v, cols ci)  -> the B operand of dx^T = A_k^T H_k^T
//   S_k = H_k    (rows ci, cols v)  -> the A operand of dA_k = H_k^T f(BN1(x))
// An MFMA accumulator holds, per lane, one column and 16 rows; read as an
// operand, those 16 rows are the k-dimension of two 16-deep k-steps in the
// order perm(hi, j) = (j & 3) + 8 (j >> 2) + 4 hi (+ 16 ks). The A image (dx
// A operand) and the f(BN1(x)) image (dA B operand) are laid out in the same
// order, so H goes from the channel GEMM's accumulators straight into the joint
// contractions without a transpose or an LDS round trip.
// Per item: dZ in chunks of CR channels (rounded to bf16, [frame][v][r] image,
// double-buffered; the next chunk -- or the next item's first chunk and its x
// slice -- loaded under this chunk's MFMAs), packed bf16 W' chunk by LDS-DMA;
// dx^T partials into an LDS row image; the row pass (16 threads per channel)
// applies the ReLU mask, accumulates the BN1 sums and stores dx coalesced.
// Numerics (the bf16 path's, as k_spatial_bwd6<.., BF = true>): H from bf16 dZ
// and W' with fp32 accumulation (the unfused bf16 H GEMM's roundings), then
// H and A to 2^-16 (h + m bf16 planes, three products) in dx, H to 2^-16 and
// f(BN1(x)) to bf16 (two products) in dA; BN1 sums in fp32 / fp64.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "internal.h"

namespace stgcn {

typedef __bf16 spb_bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 spb_bf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned spb_pk(float a, float b) {
  const spb_bf2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}
// (a, b) -> packed bf16 h and bf16 of the residual m (a == h + m to 2^-16)
__device__ __forceinline__ void spb_split(float a, float b, unsigned &h, unsigned &m) {
  h = spb_pk(a, b);
  m = spb_pk(a - __builtin_bit_cast(float, h << 16),
             b - __builtin_bit_cast(float, h & 0xffff0000u));
}
__device__ __forceinline__ floatx16 spb_mfma(uint4 a, uint4 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(spb_bf8, a),
                                                 __builtin_bit_cast(spb_bf8, b), c, 0, 0, 0);
}

template <int V, int K>
struct SpBwdGeo {
  static constexpr int NVT = (V + 31) / 32;         // 32-joint tiles (v and w)
  static constexpr int FT = 8 / NVT;                // frames per item (wave = frame, v tile)
  static constexpr int NPOS = FT * V;               // positions per item
  static constexpr int CB = 32;                     // input channels per item
  static constexpr int CR = 16;                     // dZ channels per chunk
  static constexpr int KSC = CR / 16;               // MFMA k-steps per chunk
  static constexpr int VR = NVT * 32;               // image rows per frame (joints, padded)
  static constexpr int DZP = (CR + 8) * 2;          // dZ image row pitch, bytes (b128 conflict-free)
  static constexpr int DZ_BYTES = FT * VR * DZP;
  static constexpr int W_BYTES = K * CR * 64;       // W' chunk [k][octet][ci 32][8] bf16
  static constexpr int XBP = 80;                    // f(BN1(x)) image row pitch, bytes
  static constexpr int XB_BYTES = FT * VR * XBP;
  static constexpr int AIMG_BYTES = K * NVT * NVT * 2 * 2 * 1024;  // [k][vt][wt][ks][plane] 1 KiB
  static constexpr int SP = NPOS + 1;               // dx row image pitch (floats, odd)
  static constexpr int ST_BYTES = (CB * SP * 4 + 15) & ~15;
  static constexpr int DRED_BYTES = (K * V * V * 4 + 1023) & ~1023;
  static constexpr int NDZ = NPOS * (CR / 8);       // dZ staging items (octet, position)
  static constexpr int DZIPT = (NDZ + 511) / 512;
  static constexpr int NX = NPOS * (CB / 8);        // x staging items
  static constexpr int XIPT = (NX + 511) / 512;
  static constexpr int OFF_A = 0, OFF_DZ = AIMG_BYTES, OFF_W = OFF_DZ + 2 * DZ_BYTES;
  static constexpr int OFF_XB = OFF_W + 2 * W_BYTES, OFF_ST = OFF_XB + XB_BYTES;
  static constexpr int OFF_DRED = OFF_ST + ST_BYTES;
  static constexpr int OFF_BN = OFF_DRED + DRED_BYTES;  // [2][mean | a | beta][32] floats
  static constexpr int LDS = OFF_BN + 2 * 3 * 32 * 4;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(W_BYTES % 1024 == 0 && AIMG_BYTES % 1024 == 0, "whole DMA rounds");
};

struct SpBwdParams {
  const float *dZ, *x, *mean, *invstd, *g, *b;
  const __bf16 *wpk;   // [cb][chunk][k][octet][ci 32][8]
  const __bf16 *aimg;  // [k][vt][wt][ks][plane][lane][8]
  float *dx, *dA;
  double *sd, *sdn;
  int C, R, T, ncb, nft, nitems, write_dx, relu;
};

template <int V, int K>
__global__ __launch_bounds__(512, 1) void k_sp_bwd_fused(SpBwdParams P) {
  using G = SpBwdGeo<V, K>;
  constexpr int NVT = G::NVT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int f = wave / NVT, vt = wave % NVT;  // this wave's frame and joint tile
  const int TV = P.T * V;
  const int NCH = P.R / G::CR;
  const int NG = gridDim.x;

  // ---- prologue: zero the images (pad rows stay zero), A image by LDS-DMA
  for (int e = tid; e < (2 * G::DZ_BYTES) / 16; e += 512)
    reinterpret_cast<uint4 *>(lds + G::OFF_DZ)[e] = make_uint4(0u, 0u, 0u, 0u);
  for (int e = tid; e < G::XB_BYTES / 16; e += 512)
    reinterpret_cast<uint4 *>(lds + G::OFF_XB)[e] = make_uint4(0u, 0u, 0u, 0u);
  for (int e = tid; e < G::DRED_BYTES / 4; e += 512) reinterpret_cast<float *>(lds + G::OFF_DRED)[e] = 0.f;
  {
    const __amdgpu_buffer_rsrc_t ra =
        make_rsrc(reinterpret_cast<const float *>(P.aimg), G::AIMG_BYTES / 4);
    for (int i = wave; i < G::AIMG_BYTES / 1024; i += 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, smem + i * 256, 16,
                                               (unsigned)(i * 1024 + lane * 16), 0, 0, 0);
  }

  const __amdgpu_buffer_rsrc_t rw =
      make_rsrc(reinterpret_cast<const float *>(P.wpk), (int64_t)P.ncb * NCH * G::W_BYTES / 4);
  auto dma_w = [&](int cb, int c, int buf) {
    const unsigned src = (unsigned)((cb * NCH + c) * G::W_BYTES);
    for (int i = wave; i < G::W_BYTES / 1024; i += 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rw, reinterpret_cast<float *>(lds + G::OFF_W + buf * G::W_BYTES + i * 1024), 16,
          src + (unsigned)(i * 1024 + lane * 16), 0, 0, 0);
  };
  // dZ chunk: items (octet o of the chunk's channels, position); 8 channels per item
  float dzr[G::DZIPT][8];
  auto load_dz = [&](int n, int ft, int c) {
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc(P.dZ + (int64_t)n * P.R * TV, (int64_t)P.R * TV);
    const int p0 = ft * G::FT * V;
#pragma unroll
    for (int k = 0; k < G::DZIPT; ++k) {
      const int e = k * 512 + tid;
      const int o = e / G::NPOS, pos = e - o * G::NPOS;
      const bool ok = e < G::NDZ && p0 + pos < TV;
      const int off = ((c * G::CR + 8 * o) * TV + p0 + pos) * 4;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        dzr[k][j] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rs, ok ? off + j * TV * 4 : (int)kOOB, 0, 0));
    }
  };
  auto write_dz = [&](int buf) {
#pragma unroll
    for (int k = 0; k < G::DZIPT; ++k) {
      const int e = k * 512 + tid;
      if (e < G::NDZ) {
        const int o = e / G::NPOS, pos = e - o * G::NPOS;
        const int fr = pos / V, v = pos - fr * V;
        uint4 w;
        w.x = spb_pk(dzr[k][0], dzr[k][1]);
        w.y = spb_pk(dzr[k][2], dzr[k][3]);
        w.z = spb_pk(dzr[k][4], dzr[k][5]);
        w.w = spb_pk(dzr[k][6], dzr[k][7]);
        *reinterpret_cast<uint4 *>(lds + G::OFF_DZ + buf * G::DZ_BYTES +
                                   (fr * G::VR + v) * G::DZP + o * 16) = w;
      }
    }
  };
  // x slice of an item: items (octet of the 32 channels, position)
  float xr[G::XIPT][8];
  auto load_x = [&](int n, int ft, int cb) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(P.x + (int64_t)n * P.C * TV, (int64_t)P.C * TV);
    const int p0 = ft * G::FT * V;
#pragma unroll
    for (int k = 0; k < G::XIPT; ++k) {
      const int e = k * 512 + tid;
      const int o = e / G::NPOS, pos = e - o * G::NPOS;
      const bool ok = e < G::NX && p0 + pos < TV;
      const int off = ((cb * G::CB + 8 * o) * TV + p0 + pos) * 4;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        xr[k][j] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rs, ok ? off + j * TV * 4 : (int)kOOB, 0, 0));
    }
  };
  float *bnt = reinterpret_cast<float *>(lds + G::OFF_BN);
  auto bn_table = [&](int cb, int slot) {
    if (tid < G::CB) {
      const int c = cb * G::CB + tid;
      bnt[slot * 96 + tid] = P.mean[c];
      bnt[slot * 96 + 32 + tid] = P.invstd[c] * P.g[c];
      bnt[slot * 96 + 64 + tid] = P.b[c];
    }
  };
  // f(BN1(x)) in bf16 at image row (frame, w), slot 16 ks + 8 hi + j for channel
  // 16 ks + perm(hi, j): channel 8 o + jj -> slot 16 (o >> 1) + 8 (jj >> 2) + 4 (o & 1) + (jj & 3)
  auto write_x = [&](int ft, int slot) {
    const float *tb = bnt + slot * 96;
    const int p0 = ft * G::FT * V;
#pragma unroll
    for (int k = 0; k < G::XIPT; ++k) {
      const int e = k * 512 + tid;
      if (e < G::NX) {
        const int o = e / G::NPOS, pos = e - o * G::NPOS;
        const int fr = pos / V, w = pos - fr * V;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ci = 8 * o + j;
          float bn = (xr[k][j] - tb[ci]) * tb[32 + ci] + tb[64 + ci];
          if (P.relu) bn = fmaxf(bn, 0.f);
          v[j] = p0 + pos < TV ? bn : 0.f;
        }
        char *row = lds + G::OFF_XB + (fr * G::VR + w) * G::XBP + (16 * (o >> 1) + 4 * (o & 1)) * 2;
        *reinterpret_cast<uint2 *>(row) = make_uint2(spb_pk(v[0], v[1]), spb_pk(v[2], v[3]));
        *reinterpret_cast<uint2 *>(row + 16) = make_uint2(spb_pk(v[4], v[5]), spb_pk(v[6], v[7]));
      }
    }
  };

  floatx16 T[K], S[K];
  floatx16 dacc[NVT == 1 ? K : 1];  // dA tiles of this wave (V <= 32: resident)
#pragma unroll
  for (int k = 0; k < (NVT == 1 ? K : 1); ++k)
#pragma unroll
    for (int i = 0; i < 16; ++i) dacc[k][i] = 0.f;
  float *st = reinterpret_cast<float *>(lds + G::OFF_ST);
  float *dred = reinterpret_cast<float *>(lds + G::OFF_DRED);

  int item = xcd_remap(blockIdx.x, NG);
  auto decode = [&](int it, int &n, int &ft, int &cb) {
    cb = it % P.ncb;
    const int r = it / P.ncb;
    ft = r % P.nft;
    n = r / P.nft;
  };
  if (item < P.nitems) {
    int n, ft, cb;
    decode(item, n, ft, cb);
    bn_table(cb, 0);
    load_x(n, ft, cb);
    load_dz(n, ft, 0);
    dma_w(cb, 0, 0);
  }
  __syncthreads();  // zeroed images, A image, BN table, first loads landed
  if (item < P.nitems) {
    int n, ft, cb;
    decode(item, n, ft, cb);
    write_dz(0);
    write_x(ft, 0);
  }
  __syncthreads();

  int gc = 0;  // chunk counter across items: image buffer gc & 1
  for (int it = 0; item < P.nitems; ++it, item += NG) {
    int n, ft, cb;
    decode(item, n, ft, cb);
    const int nxt = item + NG;
    const bool has_next = nxt < P.nitems;
    int nn = 0, nft = 0, ncb = 0;
    if (has_next) {
      decode(nxt, nn, nft, ncb);
      bn_table(ncb, (it + 1) & 1);  // read after the post-dA barrier
    }
    if constexpr (NVT > 1) {  // dx partials of the joint tiles meet by LDS atomics
      for (int e = tid; e < G::CB * G::SP; e += 512) st[e] = 0.f;
      if (NCH == 1) __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int i = 0; i < 16; ++i) T[k][i] = S[k][i] = 0.f;

    // ---- H_k = W_k^T dZ in both orientations, over chunks of CR channels of dZ
    for (int c = 0; c < NCH; ++c, ++gc) {
      const int buf = gc & 1;
      if (c + 1 < NCH) {
        load_dz(n, ft, c + 1);
        dma_w(cb, c + 1, buf ^ 1);
      } else if (has_next) {
        load_dz(nn, nft, 0);
        dma_w(ncb, 0, buf ^ 1);
      }
      const char *dz = lds + G::OFF_DZ + buf * G::DZ_BYTES + (f * G::VR + vt * 32 + lo) * G::DZP + hi * 16;
      const char *wb = lds + G::OFF_W + buf * G::W_BYTES + hi * 512 + lo * 16;
#pragma unroll
      for (int ks = 0; ks < G::KSC; ++ks) {
        const uint4 a = *reinterpret_cast<const uint4 *>(dz + ks * 32);
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const uint4 w = *reinterpret_cast<const uint4 *>(wb + k * (G::CR / 8) * 512 + ks * 1024);
          T[k] = spb_mfma(a, w, T[k]);  // [v][ci] = sum_r dZ[r][v] W_k[r][ci]
          S[k] = spb_mfma(w, a, S[k]);  // [ci][v]
        }
      }
      if (c + 1 < NCH) {
        write_dz(buf ^ 1);
        __syncthreads();  // chunk c + 1 in LDS; every wave is done with chunk c
      }
    }

    // ---- dx^T[w][ci] = sum_k sum_v A_k[v][w] H_k^T[v][ci] (this wave's joint tile vt)
    {
      floatx16 dxa[NVT];
#pragma unroll
      for (int wt = 0; wt < NVT; ++wt)
#pragma unroll
        for (int i = 0; i < 16; ++i) dxa[wt][i] = 0.f;
      const char *aim = lds + G::OFF_A + lane * 16;
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          uint4 bh, bm;
          spb_split(T[k][8 * ks + 0], T[k][8 * ks + 1], bh.x, bm.x);
          spb_split(T[k][8 * ks + 2], T[k][8 * ks + 3], bh.y, bm.y);
          spb_split(T[k][8 * ks + 4], T[k][8 * ks + 5], bh.z, bm.z);
          spb_split(T[k][8 * ks + 6], T[k][8 * ks + 7], bh.w, bm.w);
#pragma unroll
          for (int wt = 0; wt < NVT; ++wt) {
            const char *ab = aim + ((((k * NVT + vt) * NVT + wt) * 2 + ks) * 2) * 1024;
            const uint4 ah = *reinterpret_cast<const uint4 *>(ab);
            const uint4 am = *reinterpret_cast<const uint4 *>(ab + 1024);
            dxa[wt] = spb_mfma(ah, bh, dxa[wt]);
            dxa[wt] = spb_mfma(am, bh, dxa[wt]);
            dxa[wt] = spb_mfma(ah, bm, dxa[wt]);
          }
        }
      // lane = channel lo, rows = joints w: into the dx row image [ci][f*V + w]
#pragma unroll
      for (int wt = 0; wt < NVT; ++wt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int w = wt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
          if (w < V) {
            float *dst = st + lo * G::SP + f * V + w;
            if constexpr (NVT == 1)
              *dst = dxa[wt][i];
            else
              atomicAdd(dst, dxa[wt][i]);
          }
        }
    }
    // the next item's x slice (issued here, after the H^T tiles retired: registers)
    if (has_next) load_x(nn, nft, ncb);
    // ---- dA_k[v][w] += sum_ci H_k[ci][v] f(BN1(x))[ci][w] (this frame's 32 channels)
    {
      const char *xb = lds + G::OFF_XB + (f * G::VR + lo) * G::XBP + hi * 16;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        uint4 sh[2], sm[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          spb_split(S[k][8 * ks + 0], S[k][8 * ks + 1], sh[ks].x, sm[ks].x);
          spb_split(S[k][8 * ks + 2], S[k][8 * ks + 3], sh[ks].y, sm[ks].y);
          spb_split(S[k][8 * ks + 4], S[k][8 * ks + 5], sh[ks].z, sm[ks].z);
          spb_split(S[k][8 * ks + 6], S[k][8 * ks + 7], sh[ks].w, sm[ks].w);
        }
        if constexpr (NVT == 1) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const uint4 xv = *reinterpret_cast<const uint4 *>(xb + ks * 32);
            dacc[k] = spb_mfma(sh[ks], xv, dacc[k]);
            dacc[k] = spb_mfma(sm[ks], xv, dacc[k]);
          }
        } else {
#pragma unroll
          for (int wt = 0; wt < NVT; ++wt) {
            floatx16 d;
#pragma unroll
            for (int i = 0; i < 16; ++i) d[i] = 0.f;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              const uint4 xv = *reinterpret_cast<const uint4 *>(xb + wt * 32 * G::XBP + ks * 32);
              d = spb_mfma(sh[ks], xv, d);
              d = spb_mfma(sm[ks], xv, d);
            }
            const int w = wt * 32 + lo;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int v = vt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
              if (v < V && w < V) atomicAdd(dred + (k * V + v) * V + w, d[i]);
            }
          }
        }
      }
    }
    __syncthreads();  // dx row image complete; the f(BN1(x)) image and chunk buffers free

    // ---- row pass: 16 threads per channel: ReLU mask, BN1 sums, dx store
    {
      const int ci = tid >> 4, part = tid & 15;
      const int c = cb * G::CB + ci;
      const int p0 = ft * G::FT * V;
      const float mu = P.mean[c], is = P.invstd[c];
      const float a = is * P.g[c], be = P.b[c];
      const int64_t base = ((int64_t)n * P.C + c) * TV + p0;
      float s = 0.f, sn = 0.f;
#pragma unroll 4
      for (int q = 0; q < (G::NPOS + 15) / 16; ++q) {
        const int pos = part + 16 * q;
        if (pos < G::NPOS && p0 + pos < TV) {
          float d = st[ci * G::SP + pos];
          const float xv = P.x[base + pos];
          const float bn = (xv - mu) * a + be;
          if (P.relu && bn <= 0.f) d = 0.f;  // ReLU'(BN1(x))
          s += d;
          sn = fmaf(d, (xv - mu) * is, sn);
          if (P.write_dx) P.dx[base + pos] = d;
        }
      }
      double ds = s, dn = sn;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        ds += __shfl_xor(ds, o, 64);
        dn += __shfl_xor(dn, o, 64);
      }
      if (part == 0) {
        atomicAdd(P.sd + c, ds);
        atomicAdd(P.sdn + c, dn);
      }
    }
    if (has_next) {
      write_dz(gc & 1);
      write_x(nft, (it + 1) & 1);
    }
    __syncthreads();  // next item's images in LDS; the dx row image free
  }

  // ---- dA: per-wave tiles -> LDS -> one global atomic per element per workgroup
  if constexpr (NVT == 1) {
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int v = (i & 3) + 8 * (i >> 2) + 4 * hi;
        if (v < V && lo < V) atomicAdd(dred + (k * V + v) * V + lo, dacc[k][i]);
      }
  }
  __syncthreads();
  for (int e = tid; e < K * V * V; e += 512) atomicAdd(P.dA + e, dred[e]);
}

// W (K*R, C) -> [cb][chunk][k][octet][ci 32][8] bf16
__global__ void k_pack_spb_w(const float *W, __bf16 *wpk, int K, int R, int C, int CR) {
  const int64_t total = (int64_t)K * R * C;
  const int nch = R / CR, no = CR / 8;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = e;
    const int jj = (int)(r % 8);
    r /= 8;
    const int ci = (int)(r % 32);
    r /= 32;
    const int o = (int)(r % no);
    r /= no;
    const int k = (int)(r % K);
    r /= K;
    const int c = (int)(r % nch);
    const int cb = (int)(r / nch);
    const int rr = c * CR + 8 * o + jj;
    wpk[e] = (__bf16)W[((int64_t)k * R + rr) * C + cb * 32 + ci];
  }
}

// A (K, V, V) -> the dx A-operand image [k][vt][wt][ks][plane h, m][lane][8]:
// lane (lo, hi), j -> A_k[v = 32 vt + 16 ks + (j & 3) + 8 (j >> 2) + 4 hi][w = 32 wt + lo]
__global__ void k_pack_spb_a(const float *A, __bf16 *img, int K, int V, int NVT) {
  const int total = K * NVT * NVT * 2 * 2 * 512;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    int r = e;
    const int j = r % 8;
    r /= 8;
    const int lane = r % 64;
    r /= 64;
    const int plane = r % 2;
    r /= 2;
    const int ks = r % 2;
    r /= 2;
    const int wt = r % NVT;
    r /= NVT;
    const int vt = r % NVT;
    const int k = r / NVT;
    const int lo = lane & 31, hi = lane >> 5;
    const int v = 32 * vt + 16 * ks + (j & 3) + 8 * (j >> 2) + 4 * hi, w = 32 * wt + lo;
    const float a = (v < V && w < V) ? A[((int64_t)k * V + v) * V + w] : 0.f;
    const __bf16 h = (__bf16)a;
    img[e] = plane == 0 ? h : (__bf16)(a - (float)h);
  }
}

bool sp_bwd_fused_supported(int C, int V, int K, int R) {
  const int CR = 16;
  // V = 50: compiled, not selected (5.4 ms per cfg5 layer vs 1.6 for the unfused
  // pair: its per-item LDS atomics and one-chunk prefetch distance are latency-bound)
  static const bool v50 = getenv("STGCN_SPB_V50") != nullptr;  // A/B only
  return (V == 25 || (V == 50 && v50)) && K == 3 && C > 0 && C % 32 == 0 && R > 0 &&
         R % CR == 0;
}

static constexpr size_t kSpbAimgMax = 3 * 2 * 2 * 2 * 2 * 1024;

size_t sp_bwd_fused_wpk_bytes(int C, int R, int K, int V) {
  (void)V;
  return kSpbAimgMax + (size_t)K * R * C * 2 + 256;
}

template <int V, int K>
static hipError_t launch_spb(const SpBwdParams &P, int grid, hipStream_t s) {
  using G = SpBwdGeo<V, K>;
  hipLaunchKernelGGL((k_sp_bwd_fused<V, K>), dim3(grid), dim3(512), G::LDS, s, P);
  return hipGetLastError();
}

hipError_t launch_sp_bwd_fused(const float *dZ, const float *x, const float *mean,
                               const float *invstd, const float *g, const float *b,
                               const float *A, const float *W, void *wpk, float *dx, float *dA,
                               double *sd, double *sdn, int N, int C, int R, int T, int V, int K,
                               int write_dx, int relu, hipStream_t s) {
  if (!sp_bwd_fused_supported(C, V, K, R)) return hipErrorInvalidValue;
  const int CR = 16, NVT = (V + 31) / 32, FT = 8 / NVT;
  __bf16 *aimg = reinterpret_cast<__bf16 *>(wpk);
  __bf16 *wp = aimg + kSpbAimgMax / 2;
  hipLaunchKernelGGL(k_pack_spb_a, dim3(24), dim3(256), 0, s, A, aimg, K, V, NVT);
  const int64_t nw = (int64_t)K * R * C;
  hipLaunchKernelGGL(k_pack_spb_w, dim3((unsigned)std::min<int64_t>((nw + 255) / 256, 1024)),
                     dim3(256), 0, s, W, wp, K, R, C, CR);
  SpBwdParams P{};
  P.dZ = dZ;
  P.x = x;
  P.mean = mean;
  P.invstd = invstd;
  P.g = g;
  P.b = b;
  P.wpk = wp;
  P.aimg = aimg;
  P.dx = dx;
  P.dA = dA;
  P.sd = sd;
  P.sdn = sdn;
  P.C = C;
  P.R = R;
  P.T = T;
  P.ncb = C / 32;
  P.nft = (T + FT - 1) / FT;
  const int64_t items = (int64_t)N * P.nft * P.ncb;
  if (items >= (int64_t)1 << 31 || (int64_t)R * T * V * 4 >= ((int64_t)1 << 31) ||
      (int64_t)C * T * V * 4 >= ((int64_t)1 << 31))
    return hipErrorInvalidValue;
  P.nitems = (int)items;
  P.write_dx = write_dx;
  P.relu = relu;
  const int grid = (int)std::min<int64_t>(items, 256);
  if (V == 25) return launch_spb<25, 3>(P, grid, s);
  return launch_spb<50, 3>(P, grid, s);
}

}  // namespace stgcn

// Fused SpatialConv backward of the bf16 path (STGCN_F_BF16) — gfx950 only.
//
// k_sp_bwd_fused<V, K>: the backward of the spatial graph convolution in the
// form (1) of capi.hip, from dZ (the gradient at the SpatialConv output,
// st_graphconv.py:139-152) to dxhat, dA and the BN1 backward sums, in ONE
// kernel, so the K*C_in-channel H = W'^T dZ never reaches HBM (the unfused
// path writes H with a channel GEMM and reads it back in k_spatial_bwd5):
//   H_k[ci][t][v]  = sum_r W_k[r][ci] dZ[r][t][v]           (channel GEMM, MFMA)
//   dxhat[ci][t][w] = sum_k sum_v H_k[ci][t][v] A_k[v][w]   (joint contraction)
//   dA_k[v][w]    += sum_{ci,t} H_k[ci][t][v] f(BN1(x))[ci][t][w]
//   sd[ci] += sum dx, sdn[ci] += sum dx * xhat (BN1 backward), dx = dxhat
//   (f = ReLU in the residual block, st_graphconv.py:72-74: dx masked where
//   BN1(x) <= 0)
// Joint counts V <= 32 (one 32-joint MFMA tile: the NTU graph, V = 25).
// Persistent grid, one 8-wave workgroup per CU; work item = (clip n, 8 frames,
// 32 input channels); wave w owns frame w of the item and computes its H tiles
// in BOTH orientations from the same operand fragments:
//   T_k = H_k^T  (rows v, cols ci)  -> the B operand of dx^T = A_k^T H_k^T
//   S_k = H_k    (rows ci, cols v)  -> the A operand of dA_k = H_k^T f(BN1(x))
// An MFMA accumulator holds, per lane, one column and 16 rows; read as an
// operand, those 16 rows are the k-dimension of two 16-deep k-steps in the
// order perm(hi, j) = (j & 3) + 8 (j >> 2) + 4 hi (+ 16 ks). The A image (dx
// A operand) and the f(BN1(x)) image (dA B operand) are laid out in that
// order, so H goes from the channel GEMM's accumulators straight into the joint
// contractions: no transpose, no LDS round trip.
// Memory pipeline: dZ in chunks of 16 channels (rows of 8 frames x V joints,
// fp32) and the packed bf16 W' chunk by LDS-DMA into a D-deep ring (chunks
// of the next item included), one barrier per chunk, waits counted by hand
// (the compiler would drain the ring at every LDS read); dZ is rounded to
// bf16 at fragment read. The item's x slice lands by LDS-DMA under the
// chunk loop; the row pass (16 threads per channel) applies the ReLU mask,
// accumulates the BN1 sums in LDS (flushed once per workgroup), stores dx
// coalesced and writes the f(BN1(x)) image for the dA contraction.
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
typedef int spb_i4 __attribute__((ext_vector_type(4)));

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
// buffer resource for inline-asm loads (base, bytes)
__device__ __forceinline__ spb_i4 spb_rsrc(const void *base, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  if (bytes > 0x7fffffffLL) bytes = 0x7fffffffLL;
  if (bytes < 0) bytes = 0;
  return spb_i4{(int)(uint32_t)a, (int)((a >> 32) & 0xffff), (int)bytes, 0x00020000};
}
// 16-byte LDS-DMA of this lane's piece: LDS[m0 + 16 lane] = mem[voff] (past the
// resource: 0).
// Inline asm so the compiler does not wait for it before unrelated LDS reads.
__device__ __forceinline__ void spb_dma16(spb_i4 rs, unsigned voff, unsigned m0v) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(m0v), "v"(voff), "s"(rs)
      : "memory");
}
// s_waitcnt vmcnt(n) for the counts this kernel uses (immediates only)
__device__ __forceinline__ void spb_wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
__device__ __forceinline__ void spb_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

#ifndef STGCN_SPB_EXP  // timing experiments only (bits skip work; results wrong)
#define STGCN_SPB_EXP 0
#endif

// (a, b) -> packed bf16 planes h, m, l (a == h + m + l exactly; kernels_x3.hip)
__device__ __forceinline__ void spb_split3(float a, float b, unsigned &h, unsigned &m,
                                           unsigned &l) {
  h = spb_pk(a, b);
  const float ra = a - __builtin_bit_cast(float, h << 16);
  const float rb = b - __builtin_bit_cast(float, h & 0xffff0000u);
  m = spb_pk(ra, rb);
  l = spb_pk(ra - __builtin_bit_cast(float, m << 16), rb - __builtin_bit_cast(float, m & 0xffff0000u));
}
// 8 floats -> operand planes (2: h, m; 3: h, m, l)
template <int NP>
__device__ __forceinline__ void spb_planes(const float (&v)[8], uint4 (&o)[NP]) {
  static_assert(NP == 2 || NP == 3, "planes");
  if constexpr (NP == 2) {
    spb_split(v[0], v[1], o[0].x, o[1].x);
    spb_split(v[2], v[3], o[0].y, o[1].y);
    spb_split(v[4], v[5], o[0].z, o[1].z);
    spb_split(v[6], v[7], o[0].w, o[1].w);
  } else {
    spb_split3(v[0], v[1], o[0].x, o[1].x, o[2].x);
    spb_split3(v[2], v[3], o[0].y, o[1].y, o[2].y);
    spb_split3(v[4], v[5], o[0].z, o[1].z, o[2].z);
    spb_split3(v[6], v[7], o[0].w, o[1].w, o[2].w);
  }
}
// sum over the split products of weight >= 2^-16 of two 3-plane operands:
// h*h into acc[0], h*m + m*h + h*l + m*m + l*h into acc[1] (kernels_x3.hip)
__device__ __forceinline__ void spb_mfma6(const uint4 (&a)[3], const uint4 (&b)[3],
                                          floatx16 (&acc)[2]) {
  acc[0] = spb_mfma(a[0], b[0], acc[0]);
  acc[1] = spb_mfma(a[0], b[1], acc[1]);
  acc[1] = spb_mfma(a[1], b[0], acc[1]);
  acc[1] = spb_mfma(a[0], b[2], acc[1]);
  acc[1] = spb_mfma(a[1], b[1], acc[1]);
  acc[1] = spb_mfma(a[2], b[0], acc[1]);
}

// X3 = false: the bf16 path (bf16 W', dZ rounded to bf16; H, A to 2^-16).
// X3 = true : the fp32 path of STGCN_F_F32X3 (every operand as its exact 3-way
//             bf16 split, six products per fp32 product, h*h accumulated apart).
// DZB: dZ is stored in bf16 (capi.hip dz_bf16; the values the fp32 path rounds
//      it to): half-size ring slots, so the ring is 6 chunks deep instead of 4.
template <int V, int K, bool X3, bool DZB = false>
struct SpBwdGeo {
  static_assert(V <= 32, "one 32-joint tile");
  static constexpr int NPLW = X3 ? 3 : 1;           // W' planes
  static constexpr int NPLA = X3 ? 3 : 2;           // A planes (dx A operand)
  static constexpr int NPLX = X3 ? 3 : 1;           // f(BN1(x)) planes (dA B operand)
  static constexpr int NACC = X3 ? 2 : 1;           // accumulators per tile (h*h apart)
  static constexpr int FT = 8;                      // frames per item (wave = frame)
  static constexpr int NPOS = FT * V;               // positions per item
  // 16-byte pieces per row: NPOS positions from a 16-byte aligned start up to 3
  // floats before the row (rows of a clip start at (channel * T * V + p0) floats)
  static constexpr int NPC = (NPOS + 3 + 3) / 4;
  static constexpr int CB = 32;                     // input channels per item
  static constexpr int CR = 16;                     // dZ channels per chunk (one k-step)
  static constexpr int D = DZB ? 6 : 4;             // ring depth (chunks)
  // row pitch (floats): whole pieces, and 8 rows apart = 32 banks apart
  static constexpr int RP = (NPC * 4) % 8 == 0 ? NPC * 4 + 4 : NPC * 4;
  static_assert(NPOS % 8 == 0, "item starts p0 16-byte aligned within a row (fp32 and bf16)");
  // the dZ ring rows: fp32 as the x slice, or bf16 (NPCZ 8-element pieces from
  // the 16-byte boundary below the row start; pitch = 8 mod 16 elements)
  static constexpr int NPCZ = DZB ? (NPOS + 7 + 7) / 8 : NPC;
  static constexpr int RPZ = DZB ? ((NPCZ * 8) % 16 == 0 ? NPCZ * 8 + 8 : NPCZ * 8) : RP;
  static constexpr int ZSZ = DZB ? 2 : 4;
  static constexpr int RING_SLOT = CR * RPZ * ZSZ;  // [r][RPZ]
  static constexpr int W_BYTES = K * NPLW * CR * 64;  // W' chunk [k][plane][octet 2][ci 32][8]
  static constexpr int WPW = W_BYTES / 16 / 8;      // W' pieces per wave
  static constexpr int XBP = 80;                    // f(BN1(x)) image row pitch, bytes
  static constexpr int XB_ROWS = NPOS + 1;          // rows (frame, w) + one zero row
  static constexpr int XB_PLANE = XB_ROWS * XBP;
  static constexpr int AIMG_BYTES = K * 2 * NPLA * 1024;  // [k][ks][plane] 1 KiB fragments
  static constexpr int SP = NPOS + 1;               // dx row image pitch (floats, odd)
  static constexpr int CMAX = 256;                  // channels of the BN tables / sums
  static constexpr int OFF_A = 0, OFF_RING = AIMG_BYTES;
  static constexpr int OFF_W = OFF_RING + D * RING_SLOT;
  static constexpr int OFF_X = OFF_W + D * W_BYTES;                        // fp32 [ci][RP]
  static constexpr int OFF_ST = OFF_X + CB * RP * 4;                        // fp32 [ci][SP]
  static constexpr int OFF_XB = (OFF_ST + CB * SP * 4 + 15) & ~15;          // bf16 image
  // [mean|invstd|a|beta][CMAX] of BN1, then (prev mode) the same of the previous block's BN2
  static constexpr int OFF_TAB = (OFF_XB + NPLX * XB_PLANE + 15) & ~15;
  static constexpr int OFF_SUM = OFF_TAB + 8 * CMAX * 4;  // [s | sn | s1 | s2][CMAX] fp64
  static constexpr int LDS = OFF_SUM + 4 * CMAX * 8;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(K * V * V * 4 <= D * RING_SLOT, "dA reduction fits the ring");
  static_assert(W_BYTES % 128 == 0 && WPW <= 64, "W' pieces per wave");
  static_assert(NPC <= 64 && NPCZ <= 64, "one DMA instruction per row");
};

struct SpBwdParams {
  const float *dZ, *x, *mean, *invstd, *g, *b;
  const __bf16 *wpk;   // [cb][chunk][k][plane][octet][ci 32][8]
  const __bf16 *aimg;  // [k][ks][plane][lane][8]
  float *dx, *dA;
  double *sd, *sdn;
  int C, R, T, ncb, nft, nitems, write_dx, relu;
  PrevBn prev;  // prev mode (internal.h): x is the previous block's U
};

template <int V, int K, bool X3, bool DZB>
__global__ __launch_bounds__(512, 1) void k_sp_bwd_fused(SpBwdParams P) {
  using G = SpBwdGeo<V, K, X3, DZB>;
  constexpr int D = G::D, NACC = G::NACC;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int f = wave;  // this wave's frame of the item
  const int TV = P.T * V;
  const int NCH = P.R / G::CR;
  const int NG = gridDim.x;
  const unsigned lds0 = (unsigned)reinterpret_cast<uintptr_t>(lds);

  // ---- prologue: BN tables of all channels, zeroed sums and zero row, A image
  float *tab = reinterpret_cast<float *>(lds + G::OFF_TAB);
  double *sums = reinterpret_cast<double *>(lds + G::OFF_SUM);
  const bool pv = P.prev.mean != nullptr;
  for (int c = tid; c < P.C; c += 512) {
    const float is = P.invstd[c];
    tab[c] = P.mean[c];
    tab[G::CMAX + c] = is;
    tab[2 * G::CMAX + c] = is * P.g[c];
    tab[3 * G::CMAX + c] = P.b[c];
    if (pv) {
      const float pis = P.prev.invstd[c];
      tab[4 * G::CMAX + c] = P.prev.mean[c];
      tab[5 * G::CMAX + c] = pis;
      tab[6 * G::CMAX + c] = pis * P.prev.g[c];
      tab[7 * G::CMAX + c] = P.prev.b[c];
    }
    sums[c] = 0.0;
    sums[G::CMAX + c] = 0.0;
    sums[2 * G::CMAX + c] = 0.0;
    sums[3 * G::CMAX + c] = 0.0;
  }
  for (int e = tid; e < G::NPLX * (G::XBP / 4); e += 512) {
    const int p = e / (G::XBP / 4), q = e - p * (G::XBP / 4);
    reinterpret_cast<unsigned *>(lds + G::OFF_XB + p * G::XB_PLANE + G::NPOS * G::XBP)[q] = 0u;
  }
  __syncthreads();  // (full drain: the table loads are ordinary loads)
  {
    const spb_i4 ra = spb_rsrc(P.aimg, G::AIMG_BYTES);
    for (int i = wave; i < G::AIMG_BYTES / 1024; i += 8)
      spb_dma16(ra, (unsigned)(i * 1024 + lane * 16), lds0 + G::OFF_A + i * 1024);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }

  // this workgroup's items: first + k * NG; global chunk g -> (item k = g / NCH, c = g % NCH)
  const int first = xcd_remap(blockIdx.x, NG);
  const int myitems = first < P.nitems ? (P.nitems - 1 - first) / NG + 1 : 0;
  const int nchunks = myitems * NCH;
  auto decode = [&](int it, int &n, int &ft, int &cb) {
    cb = it % P.ncb;
    const int r = it / P.ncb;
    ft = r % P.nft;
    n = r / P.nft;
  };
  const spb_i4 rw = spb_rsrc(P.wpk, (int64_t)P.ncb * NCH * G::W_BYTES);
  // DMA of global chunk gch (3 instructions per wave: dZ rows 2w, 2w+1 and 1/8 of W')
  auto issue_chunk = [&](int gch) {
    const int k = gch / NCH, c = gch - k * NCH;
    int n, ft, cb;
    decode(first + k * NG, n, ft, cb);
    const int p0 = ft * G::FT * V;
    const int slot = gch % D;
    const spb_i4 rz =
        DZB ? spb_rsrc(reinterpret_cast<const __bf16 *>(P.dZ) + (int64_t)n * P.R * TV,
                       (int64_t)P.R * TV * 2)
            : spb_rsrc(P.dZ + (int64_t)n * P.R * TV, (int64_t)P.R * TV * 4);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 2 * wave + h;
      const int start = (c * G::CR + r) * TV + p0;  // from the 16-byte boundary below: the row's shift
      constexpr int EPP = 16 / G::ZSZ;              // elements per 16-byte piece
      const unsigned voff = (unsigned)(((start & ~(EPP - 1)) + EPP * lane) * G::ZSZ);
      if (lane < G::NPCZ)
        spb_dma16(rz, voff, lds0 + G::OFF_RING + slot * G::RING_SLOT + r * G::RPZ * G::ZSZ);
    }
    if (lane < G::WPW)
      spb_dma16(rw, (unsigned)((cb * NCH + c) * G::W_BYTES + wave * G::WPW * 16 + lane * 16),
                lds0 + G::OFF_W + slot * G::W_BYTES + wave * G::WPW * 16);
  };
  // DMA of an item's x slice: 32 channel rows (4 per wave)
  auto issue_x = [&](int item) {
    int n, ft, cb;
    decode(item, n, ft, cb);
    const int p0 = ft * G::FT * V;
    const spb_i4 rx = spb_rsrc(P.x + (int64_t)n * P.C * TV, (int64_t)P.C * TV * 4);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int r = 4 * wave + h;
      const int start = (cb * G::CB + r) * TV + p0;
      const unsigned voff = (unsigned)(((start & ~3) + 4 * lane) * 4);
      if (lane < G::NPC) spb_dma16(rx, voff, lds0 + G::OFF_X + r * G::RP * 4);
    }
  };

  floatx16 T[K][NACC], S[K][NACC], dacc[K][NACC];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
      for (int i = 0; i < 16; ++i) dacc[k][a][i] = 0.f;
  float *st = reinterpret_cast<float *>(lds + G::OFF_ST);
  const float *xs = reinterpret_cast<const float *>(lds + G::OFF_X);

  if (myitems > 0) issue_x(first);
  for (int gch = 0; gch < D - 1 && gch < nchunks; ++gch) issue_chunk(gch);

  int gch = 0;
  for (int k = 0; k < myitems; ++k) {
    const int item = first + k * NG;
    int n, ft, cb;
    decode(item, n, ft, cb);
    const int p0 = ft * G::FT * V;
#pragma unroll
    for (int kk = 0; kk < K; ++kk)
#pragma unroll
      for (int a = 0; a < NACC; ++a)
#pragma unroll
        for (int i = 0; i < 16; ++i) T[kk][a][i] = S[kk][a][i] = 0.f;

    // ---- H_k = W_k^T dZ in both orientations, 16 channels of dZ per chunk
    for (int c = 0; c < NCH; ++c, ++gch) {
      // DMA instructions issued after chunk gch's: the ring's next chunks (3
      // each) and, in an item's first D - 1 chunks, its x slice (4, issued
      // after the previous item's row pass)
      const int after = 3 * min(D - 2, nchunks - 1 - gch) + (k > 0 && c <= D - 2 ? 4 : 0);
      spb_wait_vm(after);
      spb_barrier();  // chunk gch in LDS for every wave; chunk gch - 1 retired
      if (gch + D - 1 < nchunks) issue_chunk(gch + D - 1);
      const int slot = gch % D;
      if (STGCN_SPB_EXP & 1) continue;
      // A operand: dZ[r = 8 hi + j][frame f, joint lo] (0 past V: read at a
      // clamped joint, then selected, so the 8 reads issue back to back); row
      // 8 hi + j starts (8 hi + j) * TV mod 4 = j * TV mod 4 floats into its LDS row
      const char *wb = lds + G::OFF_W + slot * G::W_BYTES + hi * 512 + lo * 16;
      float dv[8];
      uint4 a;  // dZ rounded to bf16 (the X3 path splits dv instead)
      if constexpr (DZB) {  // stored in bf16: the same values, read as shorts
        const unsigned short *rz =
            reinterpret_cast<const unsigned short *>(lds + G::OFF_RING + slot * G::RING_SLOT) +
            8 * hi * G::RPZ + f * V + (lo < V ? lo : V - 1);
        unsigned hv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] = rz[j * G::RPZ + ((j * TV) & 7)];
#pragma unroll
        for (int j = 0; j < 8; ++j) hv[j] = lo < V ? hv[j] : 0u;
        a.x = hv[0] | (hv[1] << 16);
        a.y = hv[2] | (hv[3] << 16);
        a.z = hv[4] | (hv[5] << 16);
        a.w = hv[6] | (hv[7] << 16);
      } else {
        const float *rz =
            reinterpret_cast<const float *>(lds + G::OFF_RING + slot * G::RING_SLOT) +
            8 * hi * G::RPZ + f * V + (lo < V ? lo : V - 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) dv[j] = rz[j * G::RPZ + ((j * TV) & 3)];
#pragma unroll
        for (int j = 0; j < 8; ++j) dv[j] = lo < V ? dv[j] : 0.f;
        a.x = spb_pk(dv[0], dv[1]);
        a.y = spb_pk(dv[2], dv[3]);
        a.z = spb_pk(dv[4], dv[5]);
        a.w = spb_pk(dv[6], dv[7]);
      }
      if constexpr (!X3) {
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          const uint4 w = *reinterpret_cast<const uint4 *>(wb + kk * 1024);
          T[kk][0] = spb_mfma(a, w, T[kk][0]);  // [v][ci] = sum_r dZ[r][v] W_k[r][ci]
          S[kk][0] = spb_mfma(w, a, S[kk][0]);  // [ci][v]
        }
      } else {
        uint4 a[3];
        spb_planes<3>(dv, a);
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          uint4 w[3];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            w[p] = *reinterpret_cast<const uint4 *>(wb + (kk * 3 + p) * 1024);
          spb_mfma6(a, w, T[kk]);
          spb_mfma6(w, a, S[kk]);
        }
      }
    }

    // ---- dx^T[w][ci] = sum_k sum_v A_k[v][w] H_k^T[v][ci] -> dx row image [ci][f*V + w]
    if (!(STGCN_SPB_EXP & 2)) {
      floatx16 dxp[K][NACC];  // one chain per partition, summed at the end
#pragma unroll
      for (int kk = 0; kk < K; ++kk)
#pragma unroll
        for (int a = 0; a < NACC; ++a)
#pragma unroll
          for (int i = 0; i < 16; ++i) dxp[kk][a][i] = 0.f;
      const char *aim = lds + G::OFF_A + lane * 16;
#pragma unroll
      for (int kk = 0; kk < K; ++kk)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          float tv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            tv[j] = NACC == 2 ? T[kk][0][8 * ks + j] + T[kk][NACC - 1][8 * ks + j]
                              : T[kk][0][8 * ks + j];
          uint4 b[G::NPLA], am[G::NPLA];
          spb_planes<G::NPLA>(tv, b);
#pragma unroll
          for (int p = 0; p < G::NPLA; ++p)
            am[p] = *reinterpret_cast<const uint4 *>(aim + ((kk * 2 + ks) * G::NPLA + p) * 1024);
          if constexpr (!X3) {
            dxp[kk][0] = spb_mfma(am[0], b[0], dxp[kk][0]);
            dxp[kk][0] = spb_mfma(am[1], b[0], dxp[kk][0]);
            dxp[kk][0] = spb_mfma(am[0], b[1], dxp[kk][0]);
          } else {
            spb_mfma6(am, b, dxp[kk]);
          }
        }
      floatx16 dxa = dxp[0][0];
#pragma unroll
      for (int kk = 0; kk < K; ++kk)
#pragma unroll
        for (int a = 0; a < NACC; ++a)
          if (kk || a) dxa += dxp[kk][a];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int w = (i & 3) + 8 * (i >> 2) + 4 * hi;
        if (w < V) st[lo * G::SP + f * V + w] = dxa[i];
      }
    }
    spb_barrier();  // dx row image complete (the x slice landed with the item's chunk waits)

    // ---- row pass, 16 threads per channel: ReLU mask, BN1 sums, dx store, and
    // f(BN1(x)) into the dA operand image (row (frame, w), slot of ci; bf16 planes)
    if (!(STGCN_SPB_EXP & 4)) {
      const int ci = tid >> 4, part = tid & 15;
      const int c = cb * G::CB + ci;
      const float mu = tab[c], is = tab[G::CMAX + c];
      const float a = tab[2 * G::CMAX + c], be = tab[3 * G::CMAX + c];
      // prev mode: the x slice holds the previous block's U; x = ReLU((U - pmu) pa + pb)
      // as that block's output pass formed it, mask m = x > 0, uhat = (U - pmu) pis
      const float pmu = pv ? tab[4 * G::CMAX + c] : 0.f, pis = pv ? tab[5 * G::CMAX + c] : 1.f;
      const float pa = pv ? tab[6 * G::CMAX + c] : 1.f, pb = pv ? tab[7 * G::CMAX + c] : 0.f;
      float s1 = 0.f, s2 = 0.f;
      // slot of channel ci: 16 ks + 8 hi + j for ci = 16 ks + (j & 3) + 8 (j >> 2) + 4 hi
      const int rr = ci & 15;
      const int slot = 16 * (ci >> 4) + 8 * ((rr >> 2) & 1) + (rr & 3) + 4 * (rr >> 3);
      __bf16 *xbi = reinterpret_cast<__bf16 *>(lds + G::OFF_XB) + slot;
      float *dst = P.dx + ((int64_t)n * P.C + c) * TV + p0;
      float s = 0.f, sn = 0.f;
      constexpr int NQ = (G::NPOS + 15) / 16;
      const int nlive = min(G::NPOS, TV - p0);  // positions inside the clip
      // all reads first (branch-free: clamped positions), then the arithmetic
      float dq[NQ], xq[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int pos = min(part + 16 * q, G::NPOS - 1);
        dq[q] = st[ci * G::SP + pos];
        xq[q] = xs[ci * G::RP + ((ci * TV) & 3) + pos];
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int pos = part + 16 * q;
        const bool live = pos < nlive;
        bool pm = false;
        float uh = 0.f;
        if (pv) {
          const float t = (xq[q] - pmu) * pa + pb;
          uh = (xq[q] - pmu) * pis;
          pm = t > 0.f;
          xq[q] = pm ? t : 0.f;
        }
        const float bn = (xq[q] - mu) * a + be;
        float d = live ? dq[q] : 0.f;
        if (P.relu && bn <= 0.f) d = 0.f;  // ReLU'(BN1(x))
        s += d;
        sn = fmaf(d, (xq[q] - mu) * is, sn);
        if (pm) {
          s1 += d;
          s2 = fmaf(d, uh, s2);
        }
        if (P.write_dx && live) dst[pos] = d;
        if (pos < G::NPOS) {
          const float fx = live ? (P.relu ? fmaxf(bn, 0.f) : bn) : 0.f;
          __bf16 *xr = xbi + pos * (G::XBP / 2);  // row (frame, w) = pos
          const __bf16 h = (__bf16)fx;
          xr[0] = h;
          if constexpr (X3) {
            const float r1 = fx - (float)h;
            const __bf16 m = (__bf16)r1;
            xr[G::XB_PLANE / 2] = m;
            xr[G::XB_PLANE] = (__bf16)(r1 - (float)m);
          }
        }
      }
      double ds = s, dn = sn, d1 = s1, d2 = s2;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        ds += __shfl_xor(ds, o, 64);
        dn += __shfl_xor(dn, o, 64);
        if (pv) {
          d1 += __shfl_xor(d1, o, 64);
          d2 += __shfl_xor(d2, o, 64);
        }
      }
      if (part == 0) {  // one writer per channel per item
        sums[c] += ds;
        sums[G::CMAX + c] += dn;
        if (pv) {
          sums[2 * G::CMAX + c] += d1;
          sums[3 * G::CMAX + c] += d2;
        }
      }
    }
    spb_barrier();  // f(BN1(x)) image complete; the x slice and dx row image free
    if (k + 1 < myitems) issue_x(first + (k + 1) * NG);

    // ---- dA_k[v][w] += sum_ci H_k[ci][v] f(BN1(x))[ci][w] (this frame's 32 channels)
    if (!(STGCN_SPB_EXP & 8)) {
      const int row = lo < V ? f * V + lo : G::NPOS;  // joints past V: the zero row
      const char *xb = lds + G::OFF_XB + row * G::XBP + hi * 16;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint4 xv[G::NPLX];
#pragma unroll
        for (int p = 0; p < G::NPLX; ++p)
          xv[p] = *reinterpret_cast<const uint4 *>(xb + p * G::XB_PLANE + ks * 32);
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          float sv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            sv[j] = NACC == 2 ? S[kk][0][8 * ks + j] + S[kk][NACC - 1][8 * ks + j]
                              : S[kk][0][8 * ks + j];
          if constexpr (!X3) {
            uint4 sp[2];
            spb_planes<2>(sv, sp);
            dacc[kk][0] = spb_mfma(sp[0], xv[0], dacc[kk][0]);
            dacc[kk][0] = spb_mfma(sp[1], xv[0], dacc[kk][0]);
          } else {
            uint4 sp[3];
            spb_planes<3>(sv, sp);
            spb_mfma6(sp, xv, dacc[kk]);
          }
        }
      }
    }
  }

  // ---- flush: dA tiles -> LDS (the ring) -> one global atomic per element;
  // BN1 sums -> one global atomic per channel and workgroup
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float *dred = reinterpret_cast<float *>(lds + G::OFF_RING);
  for (int e = tid; e < K * V * V; e += 512) dred[e] = 0.f;
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < K; ++kk)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int v = (i & 3) + 8 * (i >> 2) + 4 * hi;
      const float val = NACC == 2 ? dacc[kk][0][i] + dacc[kk][NACC - 1][i] : dacc[kk][0][i];
      if (v < V && lo < V) atomicAdd(dred + (kk * V + v) * V + lo, val);
    }
  __syncthreads();
  if (myitems > 0) {
    for (int e = tid; e < K * V * V; e += 512) atomicAdd(P.dA + e, dred[e]);
    for (int c = tid; c < P.C; c += 512) {
      atomicAdd(P.sd + c, sums[c]);
      atomicAdd(P.sdn + c, sums[G::CMAX + c]);
      if (pv) {
        atomicAdd(P.prev.s1 + c, sums[2 * G::CMAX + c]);
        atomicAdd(P.prev.s2 + c, sums[3 * G::CMAX + c]);
      }
    }
  }
}

// W (K*R, C) -> [cb][chunk][k][plane][octet][ci 32][8] bf16 (16 channels of R per
// chunk; planes: bf16 rounding (NP = 1) or the exact h, m, l split (NP = 3))
__global__ void k_pack_spb_w(const float *W, __bf16 *wpk, int K, int R, int C, int NP) {
  const int64_t total = (int64_t)K * R * C * NP;
  const int nch = R / 16;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = e;
    const int jj = (int)(r % 8);
    r /= 8;
    const int ci = (int)(r % 32);
    r /= 32;
    const int o = (int)(r % 2);
    r /= 2;
    const int p = (int)(r % NP);
    r /= NP;
    const int k = (int)(r % K);
    r /= K;
    const int c = (int)(r % nch);
    const int cb = (int)(r / nch);
    const int rr = c * 16 + 8 * o + jj;
    const float w = W[((int64_t)k * R + rr) * C + cb * 32 + ci];
    const __bf16 h = (__bf16)w;
    const float r1 = w - (float)h;
    const __bf16 m = (__bf16)r1;
    wpk[e] = p == 0 ? h : (p == 1 ? m : (__bf16)(r1 - (float)m));
  }
}

// A (K, V, V) -> the dx A-operand image [k][ks][plane h, m(, l)][lane][8]:
// lane (lo, hi), j -> A_k[v = 16 ks + (j & 3) + 8 (j >> 2) + 4 hi][w = lo]
__global__ void k_pack_spb_a(const float *A, __bf16 *img, int K, int V, int NP) {
  const int total = K * 2 * NP * 512;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    int r = e;
    const int j = r % 8;
    r /= 8;
    const int lane = r % 64;
    r /= 64;
    const int plane = r % NP;
    r /= NP;
    const int ks = r % 2;
    const int k = r / 2;
    const int lo = lane & 31, hi = lane >> 5;
    const int v = 16 * ks + (j & 3) + 8 * (j >> 2) + 4 * hi, w = lo;
    const float a = (v < V && w < V) ? A[((int64_t)k * V + v) * V + w] : 0.f;
    const __bf16 h = (__bf16)a;
    const float r1 = a - (float)h;
    const __bf16 m = (__bf16)r1;
    img[e] = plane == 0 ? h : (plane == 1 ? m : (__bf16)(r1 - (float)m));
  }
}

// instantiated shapes: the NTU graph with spatial partitioning on the bf16 path
// (BASELINE cfg3) and the Kinetics graph, uniform partition, on the fp32 split
// path (cfg2)
// The fp32 split variant is compiled but not selected: at K = 1 the H tensor is
// only C_in channels and the unfused pair (fp32-MFMA H GEMM at 3.5 TB/s +
// k_spatial_bwd5) is faster (cfg2 L1 281 vs 351 us, L8 421 vs 781 us; the
// twelve split MFMAs per 16-channel chunk serialise behind each chunk's wait);
// STGCN_SPB_X3 selects it (A/B only).
bool sp_bwd_fused_supported(int C, int V, int K, int R, int T, bool x3) {
  constexpr int D = SpBwdGeo<25, 3, false>::D, CMAX = SpBwdGeo<25, 3, false>::CMAX;
  constexpr bool x3_on = STGCN_AB_SPB_X3 != 0;
  const bool shape = x3 ? (x3_on && V == 18 && K == 1) : (V == 25 && K == 3);
  return shape && C > 0 && C % 32 == 0 && C <= CMAX && R % 16 == 0 && R / 16 >= D &&
         (int64_t)std::max(R, C) * T * V * 4 < ((int64_t)1 << 31);
}

static constexpr size_t kSpbAimgBytes = 3 * 2 * 3 * 1024;

size_t sp_bwd_fused_wpk_bytes(int C, int R, int K, int V) {
  (void)V;
  return kSpbAimgBytes + (size_t)K * R * C * 2 * 3 + 256;
}

template <int V, int K, bool X3, bool DZB = false>
static hipError_t launch_spb(const SpBwdParams &P0, hipStream_t s) {
  using G = SpBwdGeo<V, K, X3, DZB>;
  SpBwdParams P = P0;
  P.nft = (P.T + G::FT - 1) / G::FT;
  const int64_t items = (int64_t)P.ncb * P.nft * P.nitems;  // (nitems: N on entry)
  if (items >= (int64_t)1 << 31) return hipErrorInvalidValue;
  P.nitems = (int)items;
  const int grid = (int)std::min<int64_t>(items, 256);
  hipLaunchKernelGGL((k_sp_bwd_fused<V, K, X3, DZB>), dim3(grid), dim3(512), G::LDS, s, P);
  return hipGetLastError();
}

hipError_t launch_sp_bwd_fused(const float *dZ, const float *x, const float *mean,
                               const float *invstd, const float *g, const float *b,
                               const float *A, const float *W, void *wpk, float *dx, float *dA,
                               double *sd, double *sdn, int N, int C, int R, int T, int V, int K,
                               int write_dx, int relu, bool x3, hipStream_t s,
                               const PrevBn *prev, int dz_bf16) {
  if (!sp_bwd_fused_supported(C, V, K, R, T, x3)) return hipErrorInvalidValue;
  const int npw = x3 ? 3 : 1, npa = x3 ? 3 : 2;
  __bf16 *aimg = reinterpret_cast<__bf16 *>(wpk);
  __bf16 *wp = aimg + kSpbAimgBytes / 2;
  hipLaunchKernelGGL(k_pack_spb_a, dim3(24), dim3(256), 0, s, A, aimg, K, V, npa);
  const int64_t nw = (int64_t)K * R * C * npw;
  hipLaunchKernelGGL(k_pack_spb_w, dim3((unsigned)std::min<int64_t>((nw + 255) / 256, 1024)),
                     dim3(256), 0, s, W, wp, K, R, C, npw);
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
  P.nitems = N;
  P.write_dx = write_dx;
  P.relu = relu;
  if (prev) P.prev = *prev;
  if (x3) return dz_bf16 ? hipErrorInvalidValue : launch_spb<18, 1, true>(P, s);
  if (dz_bf16) return launch_spb<25, 3, false, true>(P, s);
  return launch_spb<25, 3, false>(P, s);
}

}  // namespace stgcn

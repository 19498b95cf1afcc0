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
  // issue cursor: the next chunk to DMA (item ik of this workgroup, chunk ic, ring
  // slot islot); the item's dZ resource, first-row offset and W' base are formed
  // once per item (no run-time divisions per chunk)
  int ik = 0, ic = 0, islot = 0, irow = 0, iwb = 0;
  spb_i4 rz;
  auto start_item = [&]() {
    int n = 0, ft = 0, cb = 0;
    if (ik < myitems) decode(first + ik * NG, n, ft, cb);
    rz = DZB ? spb_rsrc(reinterpret_cast<const __bf16 *>(P.dZ) + (int64_t)n * P.R * TV,
                        (int64_t)P.R * TV * 2)
             : spb_rsrc(P.dZ + (int64_t)n * P.R * TV, (int64_t)P.R * TV * 4);
    irow = ft * G::FT * V;
    iwb = cb * NCH * G::W_BYTES;
  };
  start_item();
  // DMA of the cursor's chunk (3 instructions per wave: dZ rows 2w, 2w+1 and 1/8 of
  // W'), then advance the cursor
  auto issue_chunk = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 2 * wave + h;
      const int start = irow + r * TV;  // from the 16-byte boundary below: the row's shift
      constexpr int EPP = 16 / G::ZSZ;  // elements per 16-byte piece
      const unsigned voff = (unsigned)(((start & ~(EPP - 1)) + EPP * lane) * G::ZSZ);
      if (lane < G::NPCZ)
        spb_dma16(rz, voff, lds0 + G::OFF_RING + islot * G::RING_SLOT + r * G::RPZ * G::ZSZ);
    }
    if (lane < G::WPW)
      spb_dma16(rw, (unsigned)(iwb + ic * G::W_BYTES + wave * G::WPW * 16 + lane * 16),
                lds0 + G::OFF_W + islot * G::W_BYTES + wave * G::WPW * 16);
    islot = islot + 1 == D ? 0 : islot + 1;
    irow += G::CR * TV;
    if (++ic == NCH) {
      ic = 0;
      ++ik;
      start_item();
    }
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
  for (int gch = 0; gch < D - 1 && gch < nchunks; ++gch) issue_chunk();

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
      if (gch + D - 1 < nchunks) issue_chunk();
      const int slot = gch % D;
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
    {
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
    {
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
    {
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

// ---------------------------------------------------------------------------
// The two-person graph (V = 50, two 32-joint tiles), bf16 path: the SpatialConv
// backward as TWO kernels that each recompute H = W'^T dZ from dZ on MFMA and
// keep it in registers (H never reaches HBM; the unfused pair wrote H in fp32 --
// K * C_in channels, 3x dZ at C_in = C_out -- and read it back):
//   k_sp50_dx<K>: dx = sum_k H_k A_k and the BN1 backward sums (+ the deferred-dx
//                 chain's mask sums), wave = (frame f, output joint tile wt):
//                 T_k = H_k^T for both joint tiles (the B operand of
//                 dx^T = A_k^T H_k^T, lane = ci), the A image [k][wt][vt][ks]
//                 [plane] in LDS, the row pass on the accumulator registers
//                 (lane = ci, 16 joints of frame f: mask, sums, 8-byte stores).
//   k_sp50_dA<K>: dA_k += sum H_k^T f(BN1(x)), wave = (frame f, joint tile vt):
//                 S_k = H_k (the A operand, lane = v), f(BN1(x)) as a bf16 image
//                 (row (frame, w), channel slots in the accumulator order), the
//                 12 dA tiles of the workgroup resident for the whole loop.
// One 8-wave workgroup per CU each; item = (clip, 4 frames, 32 input channels),
// every item of a workgroup in the same 32-channel block (grid a multiple of the
// block count), so the per-lane BN tables and sums stay in registers. dZ chunks
// (16 channels x 4 frames x 50 joints) and the packed W' chunk move by LDS-DMA
// through a 6-deep ring that runs across items; the item's x values are loaded
// into registers under the next item's chunk loop. Every wait counts this wave's
// own vector-memory instructions (`issued`, marks per ring slot), so the ring
// stays full across the per-item phases.
// Numerics as k_sp_bwd_fused / k_spatial_bwd6<.., BF = true>: H from bf16 dZ and
// W' with fp32 accumulation, H and A to 2^-16 (h + m planes, three products) in
// dx, H to 2^-16 and f(BN1(x)) to bf16 (two products) in dA.
// ---------------------------------------------------------------------------
template <int K>
struct Sp50Geo {
  static constexpr int V = 50, FT = 4, NPOS = FT * V;         // 200 positions per item
  static constexpr int NPC = (NPOS + 3 + 3) / 4;              // 16-byte pieces per dZ row
  static constexpr int RP = (NPC * 4) % 8 == 0 ? NPC * 4 + 4 : NPC * 4;  // row pitch (floats)
  static constexpr int CB = 32, CR = 16, D = 6;               // ci per item, dZ rows per chunk, ring depth
  static constexpr int RING_SLOT = CR * RP * 4;
  static constexpr int W_BYTES = K * CR * 64;                 // W' chunk [k][octet][ci 32][8] bf16
  static constexpr int WPW = W_BYTES / 16 / 8;                // W' pieces per wave
  static constexpr int AIMG = K * 2 * 2 * 2 * 2 * 1024;       // [k][wt][vt][ks][plane] fragments
  static constexpr int XBP = 80, XB_ROWS = NPOS + 1;          // f(BN1(x)) image (+ a zero row)
  static constexpr int XB_BYTES = (XB_ROWS * XBP + 15) & ~15;
  static constexpr int NQ2 = (NPOS + 15) / 16;                // dA kernel: x values per thread
  // k_sp50_dx: A image | dZ ring | W' ring (the sum reduction reuses the ring)
  static constexpr int L1_RING = AIMG, L1_W = L1_RING + D * RING_SLOT;
  static constexpr int LDS1 = L1_W + D * W_BYTES;
  // k_sp50_dA: dZ ring | W' ring | f(BN1(x)) image (the dA reduction reuses the ring)
  static constexpr int L2_W = D * RING_SLOT, L2_XB = L2_W + D * W_BYTES;
  static constexpr int LDS2 = L2_XB + XB_BYTES;
  static_assert(LDS1 <= 160 * 1024 && LDS2 <= 160 * 1024, "LDS budget");
  static_assert(8 * 32 * 4 * 8 <= D * RING_SLOT, "sum reduction fits the ring");
  static_assert(K * V * V * 4 <= D * RING_SLOT, "dA reduction fits the ring");
  static_assert(NPC <= 64 && WPW <= 64, "one DMA instruction per row / W' piece");
};

struct Sp50Params {
  const float *dZ, *x, *mean, *invstd, *g, *b;
  const __bf16 *wpk;   // [cb][chunk][k][octet][ci 32][8]
  const __bf16 *aimg;  // [k][wt][vt][ks][plane][lane][8]
  float *dx, *dA;
  double *sd, *sdn;
  int C, R, T, ncb, nft, nitems, write_dx, relu;
  PrevBn prev;
};

// s_waitcnt vmcnt(q) for a run-time n, q = n rounded down to a multiple of 4
// (at most 60): waiting for up to 3 more instructions than asked is safe and
// keeps the dispatch to a 16-way branch tree
__device__ __forceinline__ void sp50_wait_vm(int n) {
  const int q = n < 0 ? 0 : (n > 63 ? 15 : n >> 2);
  switch (q) {
#define SP50_W(i) \
  case i: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * i) : "memory"); break;
    SP50_W(0) SP50_W(1) SP50_W(2) SP50_W(3) SP50_W(4) SP50_W(5) SP50_W(6) SP50_W(7)
    SP50_W(8) SP50_W(9) SP50_W(10) SP50_W(11) SP50_W(12) SP50_W(13) SP50_W(14) SP50_W(15)
#undef SP50_W
  }
}

// Shared chunk pipeline of the two kernels: the ring of dZ chunks (2 rows per
// wave) and W' chunks (1/8 per wave), 3 DMA instructions per wave and chunk.
template <int K>
struct Sp50Ring {
  using G = Sp50Geo<K>;
  const Sp50Params &P;
  unsigned lds0;
  int ring_off, w_off, first, NG, NCH, TV, wave, lane, myitems;
  spb_i4 rw;
  // issue cursor: the next chunk to DMA (item ik of this workgroup, chunk ic,
  // ring slot islot); the item's dZ resource, first-row offset and W' base are
  // formed once per item (no divisions per chunk)
  int ik = 0, ic = 0, islot = 0, irow = 0, iwb = 0;
  spb_i4 rz;
  __device__ Sp50Ring(const Sp50Params &P_, unsigned lds0_, int ring_off_, int w_off_, int first_,
                      int wave_, int lane_, int myitems_)
      : P(P_), lds0(lds0_), ring_off(ring_off_), w_off(w_off_), first(first_), NG(gridDim.x),
        NCH(P_.R / 16), TV(P_.T * 50), wave(wave_), lane(lane_), myitems(myitems_) {
    rw = spb_rsrc(P.wpk, (int64_t)P.ncb * NCH * G::W_BYTES);
    start_item();
  }
  __device__ void decode(int it, int &n, int &ft, int &cb) const {
    cb = it % P.ncb;
    const int r = it / P.ncb;
    ft = r % P.nft;
    n = r / P.nft;
  }
  __device__ void start_item() {
    int n = 0, ft = 0, cb = 0;
    if (ik < myitems) decode(first + ik * NG, n, ft, cb);
    rz = spb_rsrc(P.dZ + (int64_t)n * P.R * TV, (int64_t)P.R * TV * 4);
    irow = ft * G::NPOS;  // element offset of chunk ic's row 0 (rows of a chunk TV apart)
    iwb = cb * NCH * G::W_BYTES;
  }
  // DMA of the cursor's chunk (3 instructions per wave), then advance the cursor
  __device__ void issue_next() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 2 * wave + h;
      const int start = irow + r * TV;  // from the 16-byte boundary below
      if (lane < G::NPC)
        spb_dma16(rz, (unsigned)(((start & ~3) + 4 * lane) * 4),
                  lds0 + ring_off + islot * G::RING_SLOT + r * G::RP * 4);
    }
    if (lane < G::WPW)
      spb_dma16(rw, (unsigned)(iwb + ic * G::W_BYTES + wave * G::WPW * 16 + lane * 16),
                lds0 + w_off + islot * G::W_BYTES + wave * G::WPW * 16);
    islot = islot + 1 == G::D ? 0 : islot + 1;
    irow += G::CR * TV;
    if (++ic == NCH) {
      ic = 0;
      ++ik;
      start_item();
    }
  }
  // dZ fragment of joint tile vt, frame f: rows r = 8 hi + j of the chunk in
  // slot `slot`, joint 32 vt + lo (0 past V), rounded to bf16 -- the A operand
  // [row v][k r] of T = dZ^T W, or the B operand [k r][col v] of S = W^T dZ
  __device__ uint4 dz_frag(const char *lds, int slot, int f, int vt, int hi, int lo) const {
    const int v = 32 * vt + lo;
    const float *rz = reinterpret_cast<const float *>(lds + ring_off + slot * G::RING_SLOT) +
                      8 * hi * G::RP + f * 50 + (v < 50 ? v : 49);
    float dv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dv[j] = rz[j * G::RP + ((j * TV) & 3)];
#pragma unroll
    for (int j = 0; j < 8; ++j) dv[j] = v < 50 ? dv[j] : 0.f;
    uint4 a;
    a.x = spb_pk(dv[0], dv[1]);
    a.y = spb_pk(dv[2], dv[3]);
    a.z = spb_pk(dv[4], dv[5]);
    a.w = spb_pk(dv[6], dv[7]);
    return a;
  }
};

template <int K>
__global__ __launch_bounds__(512, 1) void k_sp50_dx(Sp50Params P) {
  using G = Sp50Geo<K>;
  constexpr int D = G::D;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int f = wave & 3, wt = wave >> 2;  // this wave's frame and output joint tile
  const unsigned lds0 = (unsigned)reinterpret_cast<uintptr_t>(lds);
  const int first = xcd_remap(blockIdx.x, gridDim.x);
  const int myitems =
      first < P.nitems ? (P.nitems - 1 - first) / (int)gridDim.x + 1 : 0;
  Sp50Ring<K> ring(P, lds0, G::L1_RING, G::L1_W, first, wave, lane, myitems);
  const int NCH = ring.NCH, NG = ring.NG, TV = ring.TV;
  const int nchunks = myitems * NCH;
  const bool pv = P.prev.mean != nullptr;
  // this lane's channel (every item of the workgroup is in block first % ncb)
  const int cb = first % P.ncb, c = cb * 32 + lo;
  const float mu = P.mean[c], is = P.invstd[c], ga = is * P.g[c], be = P.b[c];
  const float pmu = pv ? P.prev.mean[c] : 0.f, pis = pv ? P.prev.invstd[c] : 1.f;
  const float pa = pv ? pis * P.prev.g[c] : 1.f, pb = pv ? P.prev.b[c] : 0.f;
  {  // A image (48 KiB) by LDS-DMA
    const spb_i4 ra = spb_rsrc(P.aimg, G::AIMG);
    for (int i = wave; i < G::AIMG / 1024; i += 8)
      spb_dma16(ra, (unsigned)(i * 1024 + lane * 16), lds0 + i * 1024);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // x (prev mode: the previous block's U) of this lane's 16 (frame f, joint w)
  // positions, w = 32 wt + 8 gq + 4 hi + {0..3}: two 8-byte loads per group
  // (one dword load per value: with 8-byte loads into float2 pairs hipcc copied
  // the odd halves out of the registers before the loads had landed)
  float xr[16];
  // byte offset of the pair (group gq, half h2) of this lane in its clip's x / dx
  auto xoff = [&](int ft, int gq, int h2) -> unsigned {
    const int t = ft * G::FT + f, w = 32 * wt + 8 * gq + 4 * hi + 2 * h2;
    const bool ok = t < P.T && w < 50;
    return ok ? (unsigned)(((int64_t)c * TV + (int64_t)t * 50 + w) * 4) : kOOB;
  };
  auto load_x = [&](int item) {
    int n, ft, cbb;
    ring.decode(item, n, ft, cbb);
    const spb_i4 rx = spb_rsrc(P.x + (int64_t)n * P.C * TV, (int64_t)P.C * TV * 4);
#pragma unroll
    for (int gq = 0; gq < 4; ++gq)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const unsigned o = xoff(ft, gq, h2);
#pragma unroll
        for (int e = 0; e < 2; ++e)
          asm volatile("buffer_load_dword %0, %1, %2, 0 offen"
                       : "=v"(xr[4 * gq + 2 * h2 + e])
                       : "v"(o == kOOB ? kOOB : o + 4u * e), "s"(rx)
                       : "memory");
      }
  };

  int issued = 0;  // vector-memory instructions this wave has issued
  int mk[D - 1];   // `issued` just after the DMA of each chunk in flight (oldest first)
  int mark_x = 0;
  if (myitems > 0) {
    load_x(first);
    issued += 16;
    mark_x = issued;
  }
#pragma unroll
  for (int i = 0; i < D - 1; ++i) {
    if (i < nchunks) {
      ring.issue_next();
      issued += 3;
    }
    mk[i] = issued;
  }
  double ds = 0.0, dn = 0.0, d1 = 0.0, d2 = 0.0;
  const char *aim = lds + lane * 16;
  int gch = 0, rslot = 0;
  for (int k = 0; k < myitems; ++k) {
    const int item = first + k * NG;
    int n, ft, cbb;
    ring.decode(item, n, ft, cbb);
    floatx16 T[K][2];
#pragma unroll
    for (int kk = 0; kk < K; ++kk)
#pragma unroll
      for (int vt = 0; vt < 2; ++vt)
#pragma unroll
        for (int i = 0; i < 16; ++i) T[kk][vt][i] = 0.f;
    // ---- T_k = H_k^T = dZ^T W_k over the chunks, both joint tiles
    for (int cc = 0; cc < NCH; ++cc, ++gch) {
      sp50_wait_vm(issued - mk[0]);
      spb_barrier();  // chunk gch in LDS for every wave; chunk gch - 1 retired
#pragma unroll
      for (int i = 0; i < D - 2; ++i) mk[i] = mk[i + 1];
      if (gch + D - 1 < nchunks) {
        ring.issue_next();
        issued += 3;
      }
      mk[D - 2] = issued;
      const int slot = rslot;
      rslot = rslot + 1 == D ? 0 : rslot + 1;
      const char *wb = lds + G::L1_W + slot * G::W_BYTES + hi * 512 + lo * 16;
      const uint4 a0 = ring.dz_frag(lds, slot, f, 0, hi, lo);
      const uint4 a1 = ring.dz_frag(lds, slot, f, 1, hi, lo);
#pragma unroll
      for (int kk = 0; kk < K; ++kk) {
        const uint4 w = *reinterpret_cast<const uint4 *>(wb + kk * 1024);
        T[kk][0] = spb_mfma(a0, w, T[kk][0]);  // [v][ci] = sum_r dZ[r][v] W_k[r][ci]
        T[kk][1] = spb_mfma(a1, w, T[kk][1]);
      }
    }
    // ---- dx^T[w][ci] = sum_k sum_v A_k[v][w] H_k^T[v][ci], w in tile wt
    floatx16 dxa;
#pragma unroll
    for (int i = 0; i < 16; ++i) dxa[i] = 0.f;
#pragma unroll
    for (int kk = 0; kk < K; ++kk)
#pragma unroll
      for (int vt = 0; vt < 2; ++vt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          float tv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) tv[j] = T[kk][vt][8 * ks + j];
          uint4 bpl[2];
          spb_planes<2>(tv, bpl);
          const int fr = (((kk * 2 + wt) * 2 + vt) * 2 + ks) * 2;
          const uint4 am0 = *reinterpret_cast<const uint4 *>(aim + fr * 1024);
          const uint4 am1 = *reinterpret_cast<const uint4 *>(aim + (fr + 1) * 1024);
          dxa = spb_mfma(am0, bpl[0], dxa);
          dxa = spb_mfma(am1, bpl[0], dxa);
          dxa = spb_mfma(am0, bpl[1], dxa);
        }
    // ---- row pass on the registers: lane = channel c, joints w of frame f
    sp50_wait_vm(issued - mark_x);
    asm volatile("" : "+v"(xr[0]), "+v"(xr[1]), "+v"(xr[2]), "+v"(xr[3]), "+v"(xr[4]),
                 "+v"(xr[5]), "+v"(xr[6]), "+v"(xr[7]), "+v"(xr[8]), "+v"(xr[9]), "+v"(xr[10]),
                 "+v"(xr[11]), "+v"(xr[12]), "+v"(xr[13]), "+v"(xr[14]), "+v"(xr[15]));
    const bool tlive = ft * G::FT + f < P.T;
    float s = 0.f, sn = 0.f, s1 = 0.f, s2 = 0.f;
    float dv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int w = 32 * wt + (i & 3) + 8 * (i >> 2) + 4 * hi;
      const bool live = tlive && w < 50;
      float xv = xr[i];
      bool pm = false;
      float uh = 0.f;
      if (pv) {  // x = ReLU((U - pmu) pa + pb) as the previous block's output pass formed it
        const float t = (xv - pmu) * pa + pb;
        uh = (xv - pmu) * pis;
        pm = t > 0.f;
        xv = pm ? t : 0.f;
      }
      const float bn = (xv - mu) * ga + be;
      float d = live ? dxa[i] : 0.f;
      if (P.relu && bn <= 0.f) d = 0.f;  // ReLU'(BN1(x)) of the residual block
      dv[i] = d;
      s += d;
      sn = fmaf(d, (xv - mu) * is, sn);
      if (pm) {
        s1 += d;
        s2 = fmaf(d, uh, s2);
      }
    }
    ds += s;
    dn += sn;
    d1 += s1;
    d2 += s2;
    if (P.write_dx) {  // (dx stores: masked positions go past the clip's resource)
      const spb_i4 rdx = spb_rsrc(P.dx + (int64_t)n * P.C * TV, (int64_t)P.C * TV * 4);
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const float2 v2 = {dv[4 * gq + 2 * h2], dv[4 * gq + 2 * h2 + 1]};
          asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen"
                       :
                       : "v"(v2), "v"(xoff(ft, gq, h2)), "s"(rdx)
                       : "memory");
        }
      issued += 8;
    }
    if (k + 1 < myitems) {
      load_x(item + NG);
      issued += 16;
      mark_x = issued;
    }
  }
  // ---- BN1 sums: lanes lo and lo + 32 hold the same channel; 8 waves -> LDS -> global
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  double sv[4] = {ds, dn, d1, d2};
#pragma unroll
  for (int i = 0; i < 4; ++i) sv[i] += __shfl_xor(sv[i], 32, 64);
  double *red = reinterpret_cast<double *>(lds + G::L1_RING);
  if (hi == 0)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(wave * 32 + lo) * 4 + i] = sv[i];
  __syncthreads();
  if (myitems > 0 && tid < 32 * (pv ? 4 : 2)) {
    const int ci = tid & 31, i = tid >> 5;
    double t = 0.0;
#pragma unroll
    for (int w8 = 0; w8 < 8; ++w8) t += red[(w8 * 32 + ci) * 4 + i];
    double *dst = i == 0 ? P.sd : i == 1 ? P.sdn : i == 2 ? P.prev.s1 : P.prev.s2;
    atomicAdd(dst + cb * 32 + ci, t);
  }
}

template <int K>
__global__ __launch_bounds__(512, 1) void k_sp50_dA(Sp50Params P) {
  using G = Sp50Geo<K>;
  constexpr int D = G::D, NQ = G::NQ2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int f = wave & 3, vt = wave >> 2;  // this wave's frame and joint tile of H
  const unsigned lds0 = (unsigned)reinterpret_cast<uintptr_t>(lds);
  const int first = xcd_remap(blockIdx.x, gridDim.x);
  const int myitems =
      first < P.nitems ? (P.nitems - 1 - first) / (int)gridDim.x + 1 : 0;
  Sp50Ring<K> ring(P, lds0, 0, G::L2_W, first, wave, lane, myitems);
  const int NCH = ring.NCH, NG = ring.NG, TV = ring.TV;
  const int nchunks = myitems * NCH;
  const bool pv = P.prev.mean != nullptr;
  // row pass thread: channel ci of the block, positions part + 16 q
  const int ci = tid >> 4, part = tid & 15;
  const int cb = first % P.ncb, c = cb * 32 + ci;
  const float mu = P.mean[c], ga = P.invstd[c] * P.g[c], be = P.b[c];
  const float pmu = pv ? P.prev.mean[c] : 0.f;
  const float pa = pv ? P.prev.invstd[c] * P.prev.g[c] : 1.f, pb = pv ? P.prev.b[c] : 0.f;
  // zero row of the f(BN1(x)) image (joints past V read it)
  for (int e = tid; e < G::XBP / 4; e += 512)
    reinterpret_cast<unsigned *>(lds + G::L2_XB + G::NPOS * G::XBP)[e] = 0u;
  float xr[NQ];
  auto load_x = [&](int item) {
    int n, ft, cbb;
    ring.decode(item, n, ft, cbb);
    const spb_i4 rx = spb_rsrc(P.x + (int64_t)n * P.C * TV, (int64_t)P.C * TV * 4);
    const int64_t base = (int64_t)c * TV + (int64_t)ft * G::NPOS;
    const int live = min(G::NPOS, TV - ft * G::NPOS);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int pos = part + 16 * q;
      const unsigned off = pos < live ? (unsigned)((base + pos) * 4) : kOOB;
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen"
                   : "=v"(xr[q])
                   : "v"(off), "s"(rx)
                   : "memory");
    }
  };
  int issued = 0;
  int mk[D - 1];
  int mark_x = 0;
  if (myitems > 0) {
    load_x(first);
    issued += NQ;
    mark_x = issued;
  }
#pragma unroll
  for (int i = 0; i < D - 1; ++i) {
    if (i < nchunks) {
      ring.issue_next();
      issued += 3;
    }
    mk[i] = issued;
  }
  floatx16 dacc[K][2];
#pragma unroll
  for (int kk = 0; kk < K; ++kk)
#pragma unroll
    for (int wt = 0; wt < 2; ++wt)
#pragma unroll
      for (int i = 0; i < 16; ++i) dacc[kk][wt][i] = 0.f;
  // channel slot of ci in the image rows: 16 ks + 8 hi + j for
  // ci = 16 ks + (j & 3) + 8 (j >> 2) + 4 hi (the S accumulator's row order)
  const int rr = ci & 15;
  const int cslot = 16 * (ci >> 4) + 8 * ((rr >> 2) & 1) + (rr & 3) + 4 * (rr >> 3);
  __bf16 *xbi = reinterpret_cast<__bf16 *>(lds + G::L2_XB) + cslot;
  int gch = 0, rslot = 0;
  for (int k = 0; k < myitems; ++k) {
    const int item = first + k * NG;
    int n, ft, cbb;
    ring.decode(item, n, ft, cbb);
    floatx16 S[K];
#pragma unroll
    for (int kk = 0; kk < K; ++kk)
#pragma unroll
      for (int i = 0; i < 16; ++i) S[kk][i] = 0.f;
    // ---- S_k = H_k = W_k^T dZ over the chunks (joint tile vt)
    for (int cc = 0; cc < NCH; ++cc, ++gch) {
      sp50_wait_vm(issued - mk[0]);
      spb_barrier();
#pragma unroll
      for (int i = 0; i < D - 2; ++i) mk[i] = mk[i + 1];
      if (gch + D - 1 < nchunks) {
        ring.issue_next();
        issued += 3;
      }
      mk[D - 2] = issued;
      const int slot = rslot;
      rslot = rslot + 1 == D ? 0 : rslot + 1;
      const char *wb = lds + G::L2_W + slot * G::W_BYTES + hi * 512 + lo * 16;
      const uint4 bz = ring.dz_frag(lds, slot, f, vt, hi, lo);
#pragma unroll
      for (int kk = 0; kk < K; ++kk) {
        const uint4 w = *reinterpret_cast<const uint4 *>(wb + kk * 1024);
        S[kk] = spb_mfma(w, bz, S[kk]);  // [ci][v] = sum_r W_k[r][ci] dZ[r][v]
      }
    }
    // ---- f(BN1(x)) of the item into the image (row (frame, w) = position)
    sp50_wait_vm(issued - mark_x);
    asm volatile("" : "+v"(xr[0]), "+v"(xr[1]), "+v"(xr[2]), "+v"(xr[3]), "+v"(xr[4]),
                 "+v"(xr[5]), "+v"(xr[6]), "+v"(xr[7]), "+v"(xr[8]), "+v"(xr[9]), "+v"(xr[10]),
                 "+v"(xr[11]), "+v"(xr[12]));
    static_assert(NQ == 13, "the register pin above names 13 values");
    {
      const int live = min(G::NPOS, TV - ft * G::NPOS);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int pos = part + 16 * q;
        if (pos < G::NPOS) {
          float xv = xr[q];
          if (pv) {
            const float t = (xv - pmu) * pa + pb;
            xv = t > 0.f ? t : 0.f;
          }
          const float bn = (xv - mu) * ga + be;
          const float fx = pos < live ? (P.relu ? fmaxf(bn, 0.f) : bn) : 0.f;
          xbi[pos * (G::XBP / 2)] = (__bf16)fx;
        }
      }
    }
    spb_barrier();  // f(BN1(x)) image complete
    if (k + 1 < myitems) {
      load_x(item + NG);
      issued += NQ;
      mark_x = issued;
    }
    // ---- dA_k[v][w] += sum_ci H_k[ci][v] f(BN1(x))[ci][w], v in tile vt
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 xv[2];
#pragma unroll
      for (int wt = 0; wt < 2; ++wt) {
        const int w = 32 * wt + lo;
        const int row = w < 50 ? f * 50 + w : G::NPOS;
        xv[wt] = *reinterpret_cast<const uint4 *>(lds + G::L2_XB + row * G::XBP + hi * 16 + ks * 32);
      }
#pragma unroll
      for (int kk = 0; kk < K; ++kk) {
        float sv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) sv[j] = S[kk][8 * ks + j];
        uint4 sp[2];
        spb_planes<2>(sv, sp);
#pragma unroll
        for (int wt = 0; wt < 2; ++wt) {
          dacc[kk][wt] = spb_mfma(sp[0], xv[wt], dacc[kk][wt]);
          dacc[kk][wt] = spb_mfma(sp[1], xv[wt], dacc[kk][wt]);
        }
      }
    }
  }
  // ---- flush: dA tiles -> LDS (the ring) -> one global atomic per element
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float *dred = reinterpret_cast<float *>(lds);
  for (int e = tid; e < K * 50 * 50; e += 512) dred[e] = 0.f;
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < K; ++kk)
#pragma unroll
    for (int wt = 0; wt < 2; ++wt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int v = 32 * vt + (i & 3) + 8 * (i >> 2) + 4 * hi, w = 32 * wt + lo;
        if (v < 50 && w < 50) atomicAdd(dred + (kk * 50 + v) * 50 + w, dacc[kk][wt][i]);
      }
  __syncthreads();
  if (myitems > 0)
    for (int e = tid; e < K * 50 * 50; e += 512) atomicAdd(P.dA + e, dred[e]);
}

// A (K, 50, 50) -> the k_sp50_dx A-operand image [k][wt][vt][ks][plane h, m][lane][8]:
// lane (lo, hi), j -> A_k[v = 32 vt + 16 ks + (j & 3) + 8 (j >> 2) + 4 hi][w = 32 wt + lo]
__global__ void k_pack_sp50_a(const float *A, __bf16 *img, int K) {
  const int total = K * 2 * 2 * 2 * 2 * 512;
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
    const int vt = r % 2;
    r /= 2;
    const int wt = r % 2;
    const int k = r / 2;
    const int lo = lane & 31, hi = lane >> 5;
    const int v = 32 * vt + 16 * ks + (j & 3) + 8 * (j >> 2) + 4 * hi, w = 32 * wt + lo;
    const float a = (v < 50 && w < 50) ? A[((int64_t)k * 50 + v) * 50 + w] : 0.f;
    const __bf16 h = (__bf16)a;
    img[e] = plane == 0 ? h : (__bf16)(a - (float)h);
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
  // V = 50: the k_sp50_dx / _dA pair re-reads dZ once per 32-channel block, so it
  // is selected up to C_in = 128 (cfg5 layer timings, kbench_spb.py: L1 1241 vs
  // 1516 us for the unfused H GEMM + k_spatial_bwd6, L4 1471 vs 1507, L5 1438 vs
  // 1596, but L8 (C_in = 256) 2156 vs 1819)
  const bool shape = x3 ? (x3_on && V == 18 && K == 1)
                        : (K == 3 && (V == 25 || (V == 50 && C <= 128)));
  return shape && C > 0 && C % 32 == 0 && C <= CMAX && R % 16 == 0 && R / 16 >= D &&
         (int64_t)std::max(R, C) * T * V * 4 < ((int64_t)1 << 31);
}

// A-operand image bytes: V = 25 [k][ks][plane] (3 planes max), V = 50 [k][wt][vt][ks][plane]
static constexpr size_t kSpbAimgBytes = std::max<size_t>(3 * 2 * 3 * 1024, Sp50Geo<3>::AIMG);

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
                               const PrevBn *prev, int dz_bf16, int only) {
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
  if (V == 50) {  // the two-person graph: k_sp50_dx + k_sp50_dA (fp32 dZ only)
    if (dz_bf16 || x3) return hipErrorInvalidValue;
    using G = Sp50Geo<3>;
    hipLaunchKernelGGL(k_pack_sp50_a, dim3(48), dim3(256), 0, s, A, aimg, K);
    Sp50Params Q{};
    Q.dZ = dZ;
    Q.x = x;
    Q.mean = mean;
    Q.invstd = invstd;
    Q.g = g;
    Q.b = b;
    Q.wpk = wp;
    Q.aimg = aimg;
    Q.dx = dx;
    Q.dA = dA;
    Q.sd = sd;
    Q.sdn = sdn;
    Q.C = C;
    Q.R = R;
    Q.T = T;
    Q.ncb = C / 32;
    Q.nft = (T + G::FT - 1) / G::FT;
    const int64_t items = (int64_t)Q.ncb * Q.nft * N;
    if (items >= (int64_t)1 << 31) return hipErrorInvalidValue;
    Q.nitems = (int)items;
    Q.write_dx = write_dx && dx != nullptr;
    Q.relu = relu;
    if (prev) Q.prev = *prev;
    // (the grid is a multiple of the channel-block count ncb = C / 32, so every
    // item of a workgroup -- first, first + grid, ... -- is in block first % ncb:
    // 255 at ncb = 3 (C_in = 96); items is itself a multiple of ncb)
    const int grid = (int)std::min<int64_t>(items, 256 / Q.ncb * Q.ncb);
    if (only != 2) hipLaunchKernelGGL((k_sp50_dx<3>), dim3(grid), dim3(512), G::LDS1, s, Q);
    if (only != 1) hipLaunchKernelGGL((k_sp50_dA<3>), dim3(grid), dim3(512), G::LDS2, s, Q);
    return hipGetLastError();
  }
  if (x3) return dz_bf16 ? hipErrorInvalidValue : launch_spb<18, 1, true>(P, s);
  if (dz_bf16) return launch_spb<25, 3, false, true>(P, s);
  return launch_spb<25, 3, false>(P, s);
}

}  // namespace stgcn

// Persistent halo-tile 3x3 / stride-1 / SAME convolution for 64-channel NHWC bf16 layers (the ResNet-18
// stage-1 convs: 56x56x64 -> 56x56x64, forward and input gradient).  SURVEY.md §2.4 N1; the reference
// triggers these through Keras Conv2D layers (no native code of its own).
//
// Why not the implicit GEMM of layers.hip: there every 64x64 output tile re-gathers its im2col rows (each
// input pixel 9 times) and re-reads the whole 64x576 weight matrix through LDS-DMA — 147 KB per tile for
// 2.4 M MAC (16 MAC/B), which bounds the stage-1 convs at ~37 us (≈ 48 GB/s per CU of LDS-DMA) against a
// ~6 us MFMA floor.  Here one workgroup per CU (1 x 256 threads, 131 KB of LDS):
//   * keeps the WHOLE weight tensor [9 taps][64 co][64 ci] (72 KB) resident in LDS for its lifetime;
//   * walks a contiguous run of output tiles (2 image rows x W pixels x 64 co), holding the input rows in
//     an 8-slot LDS ring: consecutive tiles share 2 of their 4 halo rows, so a tile loads only 2 new input
//     rows (14 KB at W = 56) by LDS-DMA (buffer_load ... lds), issued one tile ahead (zero rows above /
//     below the image come from the buffer range check; the two zero padding columns are never written);
//   * runs the 9 taps x 2 channel halves as 18 k-steps of v_mfma_f32_16x16x32_bf16 straight out of the
//     ring (no im2col at all: a tap is an address offset into the halo): 139 MAC per loaded byte.
// Operands: A = weights (rows = output channels), B = activations (columns = pixels), so the 16x16
// accumulator of a lane holds 4 CONSECUTIVE channels of one pixel: the epilogue is one 8-byte store per
// lane and block (no LDS transpose), and the per-channel BatchNorm statistics of the stored (bf16-rounded)
// outputs stay in registers across the workgroup's tiles (one f64 atomic pair per channel and wave at
// the end, into kStatSlots interleaved slots like the implicit GEMM's epilogue).
// The same kernel is the input gradient of such a layer: dX = conv(dY, W') with W'[tap][ci][co] =
// W[8 - tap][ci][co] (the HWIO shadow read with flipped taps), optionally accumulated into dX.
//
// LDS images: 16-byte chunk q of a 128-byte row r (weight row r = output channel, ring row r = halo
// column) lives at physical chunk q ^ ((r >> 1) & 7): the 16-lane groups of every ds_read_b128 below
// then touch 16 distinct bank quads.  Ring slots are (W + 2) * 128 + 64 bytes apart (the 64-byte shift
// keeps a fragment that straddles two image rows conflict-free too).
#include "tde_common.h"

#include <type_traits>

namespace tde {
namespace halo {

constexpr int kC = 64;               // input and output channels
constexpr int kPix = 128;            // bytes per pixel row (64 bf16)
constexpr int kWBytes = 9 * 64 * kPix;
constexpr int kSlots = 8;            // BN statistic slots (layers.hip kStatSlots)

struct Args {
  const bf16* x;       // [B,H,W,64] (forward: the input; input gradient: dY)
  const bf16* w;       // weights, element (tap, n, k) at w[tap' * wst + n * wsn + k], tap' = flip ? 8 - tap : tap
  long long wst, wsn;
  int flip;
  bf16* y;             // [B,H,W,64] output (forward: Y; input gradient: dX)
  int accum;           // y += result
  double* colstats;    // [kSlots][2][64] sum / sum of squares of the stored values, or null
  int B, H, W;
  int x_bytes;         // B*H*W*128 (< 2^31: the buffer resource range)
  long long* stamps;   // diagnostic phase clock (tde_halo_stamps), null in production
};

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }
// MFMA column j -> pixel of its 16-pixel block.  A ds_read_b128 serves lanes {0-3,12-15} with {20-27} (and
// {4-11} with {16-19,28-31}) in one LDS cycle: the first set reads logical chunk L (columns j = 0-3,
// 12-15), the second chunk L+1 (columns 4-11).  Giving the first set the even pixels and the second the odd
// ones puts the two sets in different 128-byte halves of the 256-byte bank row for ANY halo shift (tap
// column kw, block start), and the (r >> 1) & 7 swizzle spreads each set over its half: conflict-free
// except where a block straddles two image rows (bench/halo_micro.py; 2-way on 8 % of the reads at W=56).
__device__ __forceinline__ int pcol_perm(int j) { return j < 4 ? 2 * j : (j >= 12 ? 2 * j - 16 : 2 * j - 7); }

struct Rsrc {
#if defined(__HIP_DEVICE_COMPILE__)
  __amdgpu_buffer_rsrc_t r;
#endif
};
__device__ __forceinline__ Rsrc make_rsrc(const void* base, int bytes) {
  Rsrc b;
#if defined(__HIP_DEVICE_COMPILE__)
  b.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
#endif
  return b;
}
// 16-byte LDS-DMA load: lane i lands at lds + 16 i; offsets at or past the range read zeros
__device__ __forceinline__ void dma16(const Rsrc& b, char* lds, int voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(b.r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
#endif
}
template <int N>
__device__ __forceinline__ void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// TR image rows per tile (TR * W <= 16 * 2 * PB pixels); the 4 waves form a 2 x 2 grid: wave (wp, wc) owns
// pixel blocks PB*wp .. PB*wp + PB-1 of the tile and output-channel blocks 2wc, 2wc + 1, so per k-step
// 2 weight + PB activation fragment reads feed 2 * PB MFMAs (PB = 7 at 4 rows x 56: no padded block).
// The ring holds 2 TR + 4 rows: the current tile's TR + 2 and up to TR + 2 prefetched ones.
// The epilogue of tile t (bf16 conversion, BN statistics, 8-byte stores, the accumulated form's add) runs
// inside tile t + 1's k-loop, one (channel block, pixel block) pair per k-step, while that step's MFMAs
// are in flight: the two accumulator sets ping-pong by unrolling the tile loop twice.
// With one wave per SIMD, a wave issues in order: the VALU / LDS work of a k-step only hides under the
// matrix pipe when it sits BETWEEN the step's MFMAs (each MFMA occupies the pipe ~16 cycles).  The k loop
// is therefore one branch-free basic block (ACC = accumulate and ALLV = every pixel block valid are
// template parameters; the first tile, which has no epilogue to fold, is a separate instantiation of the
// loop) and each step is laid out by sched_group_barrier as MFMA / LDS read / 2 VALU, repeated.
template <int TR, int PB, bool ACC, bool ALLV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void conv3x3_kernel(Args a) {
  constexpr int RING = 2 * TR + 4;
  constexpr int NE = 2 * PB;  // epilogue pairs per tile (<= 18 k-steps)
  static_assert(NE <= 18, "one epilogue pair per k-step");
  extern __shared__ __attribute__((aligned(16))) unsigned char hsm[];
  char* const wl = reinterpret_cast<char*>(hsm);
  char* const ring = wl + kWBytes;
  const int W = a.W, H = a.H;
  const int SS = (W + 2) * kPix + 64;
  const int TRW = TR * W;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wp = wave >> 1, wc = wave & 1;
  const int tpi = H / TR;  // tiles per image
  const int ntiles = a.B * tpi;
  const int G = gridDim.x, g = blockIdx.x;
  const int t0 = (int)((long long)g * ntiles / G), t1 = (int)((long long)(g + 1) * ntiles / G);
  if (t0 >= t1) return;

  // ---- prologue: zero padding columns of every ring slot, weights -> LDS (swizzled)
  for (int i = tid; i < RING * 2 * 8; i += 256) {
    const int s = i >> 4, side = (i >> 3) & 1, ch = i & 7;
    *reinterpret_cast<uint4*>(ring + s * SS + (side ? (W + 1) * kPix : 0) + ch * 16) = make_uint4(0, 0, 0, 0);
  }
  stamp(a.stamps, 0);
  {  // weights by LDS-DMA: instruction (tap, 8-row group) fills rows n0 .. n0+7 of the tap; lane l lands in
     // physical chunk l % 8 of row n0 + l / 8 and so fetches logical chunk (l % 8) ^ swz(row)
    const Rsrc rw = make_rsrc(a.w, 9 * kC * kC * 2);
    const int n = (lane >> 3), p = lane & 7;
    for (int j = wave; j < 72; j += 4) {
      const int tap = j >> 3, n0 = (j & 7) * 8;
      const int st = a.flip ? 8 - tap : tap;
      const int row = n0 + n;
      dma16(rw, wl + tap * (kC * kPix) + n0 * kPix, (int)((st * a.wst + row * a.wsn + ((p ^ swz(row)) << 3)) * 2));
    }
  }

  // ---- halo rows by LDS-DMA: W/8 one-KiB instructions per row, dealt round-robin over the 4 waves
  const Rsrc rs = make_rsrc(a.x, a.x_bytes);
  const int per_row = W >> 3;
  auto issue_rows = [&](int b, int r_first, int nrows, int slot_first) {
    const int n = nrows * per_row;
    for (int j = wave; j < n; j += 4) {
      const int rr = j / per_row, jj = j - rr * per_row;
      const int r = r_first + rr;
      int slot = slot_first + rr;
      while (slot >= RING) slot -= RING;
      const int p = jj * 8 + (lane >> 3);  // image column
      const int lc = (lane & 7) ^ swz(p + 1);
      const int voff = (unsigned)r < (unsigned)H ? (((b * H + r) * W + p) * kPix + (lc << 4)) : (int)0x80000000;
      dma16(rs, ring + slot * SS + kPix + jj * 1024, voff);
    }
  };

  // ---- per-lane fragment offsets (tile invariant)
  const int q = lane >> 4, li = lane & 15;
  int aoff[2][2];  // weights: [co block][channel half]
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int n = 32 * wc + 16 * cb + li;
#pragma unroll
    for (int c = 0; c < 2; ++c) aoff[cb][c] = n * kPix + (((4 * c + q) ^ swz(n)) << 4);
  }
  bool pbv[PB];
  int prow[PB], pcol[PB], coff[PB][3][2];  // pixel block: tile row, column; [kw][channel half] column offsets
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    const int blk = PB * wp + pb;
    pbv[pb] = 16 * blk < TRW;  // wave-uniform
    int p = 16 * blk + pcol_perm(li);
    if (p >= TRW) p = 0;
    prow[pb] = p / W;
    pcol[pb] = p - prow[pb] * W;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int hc = pcol[pb] + kw;
#pragma unroll
      for (int c = 0; c < 2; ++c) coff[pb][kw][c] = hc * kPix + (((4 * c + q) ^ swz(hc)) << 4);
    }
  }
  float s1[2][4], s2[2][4];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[cb][r] = s2[cb][r] = 0.f;

  // epilogue pair e = (cb = e % 2, pb = e / 2) of a finished tile: its 4 channels of one pixel per lane
  auto epi = [&](const f32x4 (&acc)[2][PB], const bf16x4 (&old)[2][PB], const long long (&gp)[PB], int e) {
    const int cb = e & 1, pb = e >> 1;
    if (!ALLV && !pbv[pb]) return;
    float v[4] = {acc[cb][pb][0], acc[cb][pb][1], acc[cb][pb][2], acc[cb][pb][3]};
    if (ACC) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += bf2f(old[cb][pb][r]);
    }
    bf16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o[r] = f2bf(v[r]);
      const float qv = bf2f(o[r]);
      s1[cb][r] += qv;
      s2[cb][r] += qv * qv;
    }
    *reinterpret_cast<bf16x4*>(a.y + gp[pb] + 32 * wc + 16 * cb + 4 * q) = o;
  };

  f32x4 pacc[2][PB];      // the previous tile's accumulators (its epilogue runs in the next tile's k loop)
  bf16x4 pold[2][PB], old[2][PB];
  long long pgp[PB], gp[PB];
  int rbase[PB][3];
  f32x4 acc[2][PB];
  // the k loop of one tile: 18 k-steps (tap, channel half); the fragments of step s + 1 are read during
  // step s; EPI folds the previous tile's epilogue in, one pair per step
  auto kloop = [&](auto epi_on) {
    constexpr bool EPI = decltype(epi_on)::value;
    bf16x8 fa[2][2], fb[2][PB];
    auto load_step = [&](int st, bf16x8* af, bf16x8* bv) {
      const int tap = st >> 1, c = st & 1, kh = tap / 3, kw = tap - 3 * (tap / 3);
      const char* wt = wl + tap * (kC * kPix);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) af[cb] = *reinterpret_cast<const bf16x8*>(wt + aoff[cb][c]);
      // a pixel block past the tile reads pixel 0 and is never stored
#pragma unroll
      for (int pb = 0; pb < PB; ++pb) bv[pb] = *reinterpret_cast<const bf16x8*>(ring + rbase[pb][kh] + coff[pb][kw][c]);
    };
    load_step(0, fa[0], fb[0]);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      const int cur = st & 1;
      if (st + 1 < 18) load_step(st + 1, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
      for (int pb = 0; pb < PB; ++pb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) acc[cb][pb] = mfma16(fa[cur][cb], fb[cur][pb], acc[cb][pb]);
      if (EPI && st < NE) epi(pacc, pold, pgp, st);
      // lay the step out as [MFMA, LDS read, 2 VALU] x 2 PB (reads: the next step's 2 + PB fragments)
#pragma unroll
      for (int i = 0; i < 2 * PB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        if (i < 2 + PB) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // VALU
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  int s0 = 0;
  {
    const int b = t0 / tpi, r0 = TR * (t0 - b * tpi);
    issue_rows(b, r0 - 1, TR + 2, 0);
  }
  for (int t = t0; t < t1; ++t) {
    // this tile's rows have landed (DMA issued one tile ago; older stores and old-value reads long done).
    // The builtin form of the wait (not inline asm) tells the compiler's wait-count pass that nothing is
    // outstanding here, so the folded epilogue below never waits on this tile's prefetch DMA.
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_s_barrier();
    if (t == t0) stamp(a.stamps, 1);
    if (t == t0 && a.stamps && threadIdx.x == 0)  // shader-clock cycles (s_memtime) beside the 100 MHz stamps
      a.stamps[(size_t)blockIdx.x * kMaxStamps + 6] = (long long)__builtin_amdgcn_s_memtime();
    const int b = t / tpi, r0 = TR * (t - b * tpi);
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) gp[pb] = ((long long)(b * H + r0 + prow[pb]) * W + pcol[pb]) * kC;
    if (ACC) {  // the accumulated form's old values, read before the prefetch DMA is queued behind them
#pragma unroll
      for (int pb = 0; pb < PB; ++pb) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          old[cb][pb] = (ALLV || pbv[pb]) ? *reinterpret_cast<const bf16x4*>(a.y + gp[pb] + 32 * wc + 16 * cb + 4 * q)
                                          : bf16x4{};
      }
    }
    int snext = s0;
    if (t + 1 < t1) {  // prefetch the next tile's new rows into slots the current tile does not use
      const int nb = (t + 1) / tpi, nr0 = TR * ((t + 1) - nb * tpi);
      if (nb == b) {
        issue_rows(b, r0 + TR + 1, TR, s0 + TR + 2);
        snext = s0 + TR;
      } else {
        issue_rows(nb, nr0 - 1, TR + 2, s0 + TR + 2);
        snext = s0 + TR + 2;
      }
    }
#pragma unroll
    for (int pb = 0; pb < PB; ++pb)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        int sl = s0 + prow[pb] + kh;
        while (sl >= RING) sl -= RING;
        rbase[pb][kh] = sl * SS;
      }
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int pb = 0; pb < PB; ++pb) acc[cb][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t == t0) kloop(std::integral_constant<bool, false>{});
    else kloop(std::integral_constant<bool, true>{});
    if (t == t0) stamp(a.stamps, 2);
    if (t == t0 && a.stamps && threadIdx.x == 0)
      a.stamps[(size_t)blockIdx.x * kMaxStamps + 7] = (long long)__builtin_amdgcn_s_memtime();
    if (t == t0 + 1) stamp(a.stamps, 3);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int pb = 0; pb < PB; ++pb) {
        pacc[cb][pb] = acc[cb][pb];
        if (ACC) pold[cb][pb] = old[cb][pb];
      }
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) pgp[pb] = gp[pb];
    s0 = snext >= RING ? snext - RING : snext;
  }
#pragma unroll
  for (int e = 0; e < NE; ++e) epi(pacc, pold, pgp, e);
  stamp(a.stamps, 4);
  if (a.colstats) {
    // fold the two pixel-half waves of each channel half in LDS (the ring is free now), then one f64 atomic
    // pair per channel and workgroup
    __syncthreads();
    float* red = reinterpret_cast<float*>(ring);  // [wp][2 stats][64 channels]
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t1s = row16_sum(s1[cb][r]), t2s = row16_sum(s2[cb][r]);
        if (li == 0) {
          const int co = 32 * wc + 16 * cb + 4 * q + r;
          red[(wp * 2 + 0) * kC + co] = t1s;
          red[(wp * 2 + 1) * kC + co] = t2s;
        }
      }
    __syncthreads();
    if (tid < 2 * kC) {
      double* st = a.colstats + (size_t)(g % kSlots) * 2 * kC;
      atomicAdd(&st[tid], (double)(red[tid] + red[2 * kC + tid]));
    }
  }
  stamp(a.stamps, 5);
}

// ------------------------------------------------------------------------------------------------------------
// Weight gradient of the same layers: dW[tap][ci][co] = sum over pixels p of x[p + tap][ci] * dY[p][co].
// The implicit GEMM (layers.hip, register-staged at Co = 64) re-gathers every input pixel once per tap through
// L2 and runs at ~55 us per stage-1 layer for 14.8 GFLOP.  Here each workgroup (4 waves, ~147 KB of LDS) walks
// a contiguous run of tiles (TR image rows x W pixels) exactly as the convolution above does: the input rows
// with their halo in an LDS ring (TR new rows per tile, prefetched one tile ahead), the tile's dY rows in a
// double buffer, both by LDS-DMA; every input byte and dY byte is loaded ONCE for all 9 taps.
// GEMM view per tap: M = ci, N = co, K = pixels.  Both operands are pixel-major in LDS (128-byte rows of 64
// channels), so the 16x16x32 fragments (8 consecutive pixels per lane) come from CDNA4's transposed LDS read
// (ds_read_b64_tr_b16, as the weight gradients of layers.hip); a tap is an address offset into the halo ring.
// Wave w owns input channels 16w .. 16w+15 for all 9 taps and 64 output channels: 36 accumulators (144 VGPRs)
// that live across the workgroup's tiles.  Per 32-pixel k-step: 9 + 4 fragments (26 transposed reads), 36 MFMAs.
// The workgroup stores its [9][64][64] f32 partial once at the end; one reduction pass (part_reduce_kernel) sums
// the partials into the flat gradient in a fixed order (deterministic).
// LDS rows (ring columns hc, dY columns c): 16-byte chunk q of row r at physical chunk q ^ wsw(r), wsw(r) =
// (bit 1 of r, bit 3 of r) << 1 (layers.hip's RW = 64 swizzle): the 4 rows x 32 bytes of one 16-lane
// transposed read hit 16 distinct bank slots for any first row (rows r, r + 2 always differ in bit 1).
constexpr int kWgPix = 128;   // bytes per pixel row

__device__ __forceinline__ int wsw(int r) { return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1; }

typedef short wv4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) wv4 lds_wv4;
// fragment of 8 consecutive pixels (rows row0 + 8 * (lane >> 4) .. +7 of a 128-byte-row image at `base`, row r at
// base + r * 128, shifted by `rshift` rows for the swizzle) x 16 channels cb .. cb+15: lane l gets the 8 pixels
// of channel cb + (l & 15) — the A (or B) operand of v_mfma_f32_16x16x32_bf16 with K = pixels.
__device__ __forceinline__ bf16x8 wg_frag(const char* base, int row0, int cb, int lane) {
  const int i = lane & 15, q = i >> 2, pp = i & 3;
  const int r_lo = row0 + 8 * (lane >> 4) + q;
  const int ch = (cb >> 3) + (pp >> 1);
  const wv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_wv4*)(base + r_lo * kWgPix + 16 * (ch ^ wsw(r_lo)) + 8 * (pp & 1)));
  const wv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_wv4*)(base + (r_lo + 4) * kWgPix + 16 * (ch ^ wsw(r_lo + 4)) + 8 * (pp & 1)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

// 32x32x16 form: lane l gets pixels row0 + 8 * (l >> 5) .. +7 of channels cb + (l & 31) (the A / B operand of
// v_mfma_f32_32x32x16_bf16 with K = 16 pixels); each 16-lane group runs wg_frag's two transposed reads
__device__ __forceinline__ bf16x8 wg_frag32(const char* base, int row0, int cb, int lane) {
  const int i = lane & 15, q = i >> 2, pp = i & 3;
  const int r_lo = row0 + 8 * (lane >> 5) + q;
  const int ch = ((cb + 16 * ((lane >> 4) & 1)) >> 3) + (pp >> 1);
  const wv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_wv4*)(base + r_lo * kWgPix + 16 * (ch ^ wsw(r_lo)) + 8 * (pp & 1)));
  const wv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_wv4*)(base + (r_lo + 4) * kWgPix + 16 * (ch ^ wsw(r_lo + 4)) + 8 * (pp & 1)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

struct WgArgs {
  const bf16* x;    // [B,H,W,64] the layer input
  const bf16* dy;   // [B,H,W,64] the output gradient
  float* part;      // [gridDim][9][64][64] per-workgroup partial dW (HWIO order)
  int B, H, W;
  int bytes;        // B*H*W*128 (buffer range of both tensors)
};

// MF = 32: v_mfma_f32_32x32x16_bf16, wave w = input-channel half (w >> 1) x output-channel half (w & 1), 9
// accumulators of 32x32; per 16-pixel k-step 9 + 1 fragments feed 9 MFMAs (half the instructions per flop of
// the 16x16x32 form at one wave per SIMD)
template <int TR, int MF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void wgrad3x3_kernel(WgArgs a) {
  constexpr int RING = 2 * TR + 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char wsm[];
  const int W = a.W, H = a.H;
  const int SS = (W + 2) * kWgPix;          // ring slot: W + 2 halo columns
  const int DS = TR * W * kWgPix;           // dY buffer: the tile's TR rows
  char* const ring = reinterpret_cast<char*>(wsm);
  char* const dyb = ring + RING * SS;       // [2][TR * W] pixel rows
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tpi = H / TR, ntiles = a.B * tpi;
  const int G = gridDim.x, g = blockIdx.x;
  const int t0 = (int)((long long)g * ntiles / G), t1 = (int)((long long)(g + 1) * ntiles / G);

  f32x4 acc[MF == 16 ? 9 : 1][4];
  f32x16 acc2[MF == 32 ? 9 : 1];
  if constexpr (MF == 16) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc2[t][r] = 0.f;
  }

  if (t0 < t1) {
    // zero halo columns of every ring slot (never written by the DMA)
    for (int i = tid; i < RING * 2 * 8; i += 256) {
      const int sl = i >> 4, side = (i >> 3) & 1, ch = i & 7;
      *reinterpret_cast<uint4*>(ring + sl * SS + (side ? (W + 1) * kWgPix : 0) + ch * 16) = make_uint4(0, 0, 0, 0);
    }
    const halo::Rsrc rx = halo::make_rsrc(a.x, a.bytes), rd = halo::make_rsrc(a.dy, a.bytes);
    const int per_row = W >> 3;   // one-KiB DMA instructions per image row (8 pixels each)
    // input rows r_first .. (nrows of them) of image b into ring slots slot_first.. (halo column hc = p + 1);
    // rows outside the image read zeros through the range check
    auto issue_x = [&](int b, int r_first, int nrows, int slot_first) {
      const int n = nrows * per_row;
      for (int j = wave; j < n; j += 4) {
        const int rr = j / per_row, jj = j - rr * per_row;
        const int r = r_first + rr;
        int slot = slot_first + rr;
        while (slot >= RING) slot -= RING;
        const int p = jj * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ wsw(p + 1);
        const int voff = (unsigned)r < (unsigned)H ? (((b * H + r) * W + p) * kWgPix + (lc << 4)) : (int)0x80000000;
        halo::dma16(rx, ring + slot * SS + kWgPix + jj * 1024, voff);
      }
    };
    // the tile's dY rows (TR x W pixels, contiguous in memory) into dY buffer `buf` (pixel c of the tile = row c)
    auto issue_dy = [&](int b, int r0, int buf) {
      const int n = TR * per_row;
      for (int j = wave; j < n; j += 4) {
        const int c = j * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ wsw(c);
        halo::dma16(rd, dyb + buf * DS + j * 1024, ((b * H + r0) * W + c) * kWgPix + (lc << 4));
      }
    };
    int s0 = 0;
    {
      const int b = t0 / tpi, r0 = TR * (t0 - b * tpi);
      issue_x(b, r0 - 1, TR + 2, 0);
      issue_dy(b, r0, 0);
    }
    const int cb = 16 * wave;   // this wave's input channels (the A operand rows)
    for (int t = t0; t < t1; ++t) {
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_s_barrier();   // the tile's rows landed; every wave is done with the previous tile
      const int b = t / tpi, r0 = TR * (t - b * tpi);
      const int buf = (t - t0) & 1;
      int snext = s0;
      if (t + 1 < t1) {
        const int nb = (t + 1) / tpi, nr0 = TR * ((t + 1) - nb * tpi);
        if (nb == b) {
          issue_x(b, r0 + TR + 1, TR, s0 + TR + 2);
          snext = s0 + TR;
        } else {
          issue_x(nb, nr0 - 1, TR + 2, s0 + TR + 2);
          snext = s0 + TR + 2;
        }
        issue_dy(nb, nr0, buf ^ 1);
      }
      const char* dyt = dyb + buf * DS;
      if constexpr (MF == 32) {
        const int ci0 = 32 * (wave >> 1), co0 = 32 * (wave & 1);
        // k-steps of 16 pixels; lane half h = lane >> 5 takes pixels 16 k + 8 h .. +7 (one image row)
        for (int k = 0; k < TR * W / 16; ++k) {
          const int p0 = 16 * k + 8 * (lane >> 5);
          const int tr = p0 / W, c0 = p0 - tr * W;
          const bf16x8 bfr = wg_frag32(dyt, 16 * k, co0, lane);
#pragma unroll
          for (int kh = 0; kh < 3; ++kh) {
            int sl = s0 + tr + kh;
            if (sl >= RING) sl -= RING;
            const char* rowb = ring + sl * SS;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
              const bf16x8 af = wg_frag32(rowb, c0 + kw - 8 * (lane >> 5), ci0, lane);
              acc2[kh * 3 + kw] = mfma32(af, bfr, acc2[kh * 3 + kw]);
            }
          }
        }
      } else
      // k-steps of 32 pixels; lane group h = lane >> 4 takes pixels 32 k + 8 h .. +7 (one image row: W % 8 == 0)
      for (int k = 0; k < TR * W / 32; ++k) {
        const int p0 = 32 * k + 8 * (lane >> 4);
        const int tr = p0 / W, c0 = p0 - tr * W;
        bf16x8 bf[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) bf[n] = wg_frag(dyt, 32 * k, 16 * n, lane);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          int sl = s0 + tr + kh;
          if (sl >= RING) sl -= RING;
          const char* rowb = ring + sl * SS;
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            // the fragment's 8 pixels sit in ONE ring row: rows c0 + kw .. +7 (relative to this lane group);
            // wg_frag adds 8 * (lane >> 4), so pass the group-relative start minus it
            const bf16x8 af = wg_frag(rowb, c0 + kw - 8 * (lane >> 4), cb, lane);
#pragma unroll
            for (int n = 0; n < 4; ++n) acc[kh * 3 + kw][n] = mfma16(af, bf[n], acc[kh * 3 + kw][n]);
          }
        }
      }
      s0 = snext >= RING ? snext - RING : snext;
    }
  }
  float* dst = a.part + (size_t)g * 9 * 64 * 64;
  if constexpr (MF == 32) {
    // lane holds rows (ci) ci0 + 8 (r >> 2) + 4 (lane >> 5) + (r & 3), column (co) co0 + (lane & 31)
    const int w = (int)(tid >> 6), ci0 = 32 * (w >> 1), co0 = 32 * (w & 1);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = ci0 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3), co = co0 + (lane & 31);
        dst[(t * 64 + ci) * 64 + co] = acc2[t][r];
      }
  } else {
    // lane holds rows (ci) cb + 4 (lane >> 4) + r, column (co) 16 n + (lane & 15)
    const int cbs = 16 * (int)(tid >> 6);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ci = cbs + 4 * (lane >> 4) + r, co = 16 * n + (lane & 15);
          dst[(t * 64 + ci) * 64 + co] = acc[t][n][r];
        }
  }
}

// ------------------------------------------------------------------------------------------------------------
// Weight gradient of the packed RGB stem (layers.hip tde_stem_pack: the 7x7 stride-2 conv on 3 channels as a
// virtual conv over [B][Hp][Wv][8] — two real pixels x 4 channels per virtual pixel — with KWv = 4 taps along W at
// stride 1): dWv[kh][kwv][c][co] = sum over output pixels (oh, ow) of xp[oh*sh + kh][ow + kwv][c] * dY[oh][ow][co].
// The implicit GEMM (K = 802,816 pixels at batch 64) runs this at ~81 us; here, as in wgrad3x3_kernel, each
// workgroup walks tiles of TR output rows with the tile's KH + (TR-1) sh input rows and TR dY rows in LDS (LDS-DMA,
// double-buffered), every byte loaded once for all taps.  For one kh the 32 (kwv, c) rows of the A operand at
// pixel ow are the 64 contiguous bytes from virtual pixel ow: a 16-row fragment (kwv pair a) of 8 consecutive
// pixels is a transposed read of 4 overlapping 32-byte windows 16 bytes apart (each lane supplies its address).
// M = KH x 32 rows in 2 KH blocks of 16, dealt round-robin over the 4 waves; N = 64.
constexpr int kSxRow = 2048;   // LDS bytes per staged input row (<= 128 virtual pixels)

__device__ __forceinline__ bf16x8 sx_frag(const char* row, int pix0, int a, int lane) {
  const int i = lane & 15, q = i >> 2, pp = i & 3;
  const wv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_wv4*)(row + (pix0 + q + 2 * a) * 16 + pp * 8));
  const wv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_wv4*)(row + (pix0 + 4 + q + 2 * a) * 16 + pp * 8));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

struct StemWgArgs {
  const bf16* xp;   // [B][Hp][Wv][8]
  const bf16* dy;   // [B][Ho][Wo][64]
  float* part;      // [gridDim][KH * 32][64]
  int B, Hp, Wv, Ho, Wo, KH, sh;
  int x_bytes, dy_bytes;
};

template <int TR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void stem_wgrad_kernel(StemWgArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char ssm[];
  const int Wo = a.Wo, KH = a.KH, sh = a.sh;
  const int NXR = (TR - 1) * sh + KH;      // input rows of one tile
  const int XB = NXR * kSxRow, DB = TR * Wo * kWgPix;
  char* const xb = reinterpret_cast<char*>(ssm);   // [2][NXR][kSxRow]
  char* const db = xb + 2 * XB;                     // [2][TR * Wo][128]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tpi = a.Ho / TR, ntiles = a.B * tpi;
  const int G = gridDim.x, g = blockIdx.x;
  const int t0 = (int)((long long)g * ntiles / G), t1 = (int)((long long)(g + 1) * ntiles / G);
  const int NB = 2 * KH;                   // 16-row M blocks: b = 2 kh + a
  f32x4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[j][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (t0 < t1) {
    const Rsrc rx = make_rsrc(a.xp, a.x_bytes), rd = make_rsrc(a.dy, a.dy_bytes);
    const int xi = (a.Wv + 63) / 64;       // one-KiB instructions per input row
    auto issue = [&](int t, int buf) {
      const int b = t / tpi, oh0 = TR * (t - b * tpi);
      for (int j = wave; j < NXR * xi; j += 4) {
        const int r = j / xi, jj = j - r * xi;
        const int p = jj * 64 + lane;
        // pixels past the row read the next row's bytes (never used); the range check zeroes the tensor's end
        dma16(rx, xb + buf * XB + r * kSxRow + jj * 1024, ((b * a.Hp + oh0 * sh + r) * a.Wv + p) * 16);
      }
      const int per_row = Wo >> 3;
      for (int j = wave; j < TR * per_row; j += 4) {
        const int c = j * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ wsw(c);
        dma16(rd, db + buf * DB + j * 1024, ((b * a.Ho + oh0) * Wo + c) * kWgPix + (lc << 4));
      }
    };
    issue(t0, 0);
    for (int t = t0; t < t1; ++t) {
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_s_barrier();
      const int buf = (t - t0) & 1;
      if (t + 1 < t1) issue(t + 1, buf ^ 1);
      const char* xt = xb + buf * XB;
      const char* dt = db + buf * DB;
      for (int k = 0; k < TR * Wo / 32; ++k) {
        const int p0 = 32 * k + 8 * (lane >> 4);
        const int tr = p0 / Wo, ow0 = p0 - tr * Wo;
        bf16x8 bfr[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) bfr[n] = wg_frag(dt, 32 * k, 16 * n, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int b = wave + 4 * j;
          if (b < NB) {   // wave-uniform
            const int kh = b >> 1, ap = b & 1;
            const bf16x8 af = sx_frag(xt + (tr * sh + kh) * kSxRow, ow0, ap, lane);
#pragma unroll
            for (int n = 0; n < 4; ++n) acc[j][n] = mfma16(af, bfr[n], acc[j][n]);
          }
        }
      }
    }
  }
  // partial: block b rows b * 16 + 4 (lane >> 4) + r, column 16 n + (lane & 15) (dWv's flat [kh][kwv][c][co] order)
  float* dst = a.part + (size_t)g * NB * 16 * 64;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b = (int)(tid >> 6) + 4 * j;
    if (b >= NB) continue;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        dst[(b * 16 + 4 * (lane >> 4) + r) * 64 + 16 * n + (lane & 15)] = acc[j][n][r];
  }
}

// Forward of the packed RGB stem (the virtual conv of stem_wgrad_kernel: C = 8, KWv = 4 taps at stride 1, stride sh
// along H, valid, Co = 64): y[b][oh][ow][co] = sum over (kh, kwv, c) of xp[oh*sh + kh][ow + kwv][c] * Wv[co][kh][kwv][c],
// plus the BN statistics of the stored bf16 y (sum, sum of squares per channel into 8 f64 slots, as the implicit
// GEMM's epilogue).  The implicit GEMM runs this as 6,272 short-K (224) tiles, its prologue / epilogue dominating
// (~65 us); here each persistent workgroup walks tiles of TR output rows: the tile's input rows by LDS-DMA
// (double-buffered), every wave owning 16 output channels with their KH weight fragments in registers, one k-step
// per kernel row (the 32 (kwv, c) values of a pixel are the 64 contiguous bytes from its virtual pixel: a plain
// 16-byte LDS read per lane), the output tile staged in LDS and stored in coalesced 16-byte chunks.
struct StemFwdArgs {
  const bf16* xp;       // [B][Hp][Wv][8]
  const bf16* wv;       // [64][KH * 32]
  bf16* y;              // [B][Ho][Wo][64]
  double* colstats;     // [8][2][64] (nullable)
  int B, Hp, Wv, Ho, Wo, KH, sh;
  int x_bytes;
};
template <int TR>
__global__ __launch_bounds__(256) void stem_fwd_kernel(StemFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char ssm[];
  const int Wo = a.Wo, KH = a.KH, sh = a.sh;
  const int NXR = (TR - 1) * sh + KH;
  const int XB = NXR * kSxRow;
  char* const xb = reinterpret_cast<char*>(ssm);   // [2][NXR][kSxRow]
  const int tid = threadIdx.x, lane = tid & 63, fr = lane & 15, fq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tpi = a.Ho / TR, ntiles = a.B * tpi;
  const int G = gridDim.x, g = blockIdx.x;
  const int t0 = (int)((long long)g * ntiles / G), t1 = (int)((long long)(g + 1) * ntiles / G);
  // A fragments: this wave's 16 channels (rows co = 16 wave + fr), k = 32 kh + 8 fq + j
  bf16x8 wf[8];
#pragma unroll
  for (int kh = 0; kh < 8; ++kh)
    wf[kh] = kh < KH ? *reinterpret_cast<const bf16x8*>(a.wv + (size_t)(wave * 16 + fr) * (KH * 32) + kh * 32 + fq * 8)
                     : bf16x8{};
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (t0 < t1) {
    const Rsrc rx = make_rsrc(a.xp, a.x_bytes);
    const int xi = (a.Wv + 63) / 64;   // one-KiB instructions per input row
    auto issue = [&](int t, int buf) {
      const int b = t / tpi, oh0 = TR * (t - b * tpi);
      for (int j = wave; j < NXR * xi; j += 4) {
        const int r = j / xi, jj = j - r * xi;
        // pixels past the row read the next row's bytes (never used); the range check zeroes the tensor's end
        dma16(rx, xb + buf * XB + r * kSxRow + jj * 1024, ((b * a.Hp + oh0 * sh + r) * a.Wv + jj * 64 + lane) * 16);
      }
    };
    issue(t0, 0);
    for (int t = t0; t < t1; ++t) {
      __builtin_amdgcn_s_waitcnt(0);   // this tile's rows landed (and this wave's stores of the last tile drained)
      __builtin_amdgcn_s_barrier();    // ... for every wave; the other buffer is free
      const int buf = (t - t0) & 1;
      if (t + 1 < t1) issue(t + 1, buf ^ 1);
      const char* xt = xb + buf * XB;
      const int b = t / tpi, oh0 = TR * (t - b * tpi);
      bf16* yt = a.y + ((size_t)(b * a.Ho + oh0) * Wo) * 64 + wave * 16 + fq * 4;
      for (int p0 = 0; p0 < TR * Wo; p0 += 16) {
        const int tr = p0 / Wo, ow0 = p0 - tr * Wo;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 8; ++kh)
          if (kh < KH) {
            // B fragment: pixel column fr, k = 8 fq + j -> the 16 bytes at virtual pixel ow0 + fr + fq
            const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xt + (tr * sh + kh) * kSxRow + (ow0 + fr + fq) * 16);
            acc = mfma16(wf[kh], xf, acc);
          }
        // acc[r]: channel 16 wave + 4 fq + r of pixel p0 + fr: 4 consecutive channels, one 8-byte store
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = f2bf(acc[r]);
          const float v = bf2f(o[r]);
          s1[r] += v;
          s2[r] += v * v;
        }
        *reinterpret_cast<bf16x4*>(yt + (size_t)(p0 + fr) * 64) = o;
      }
    }
  }
  if (a.colstats) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[r] += __shfl_xor(s1[r], o, 64);
        s2[r] += __shfl_xor(s2[r], o, 64);
      }
    if (fr == 0 && t0 < t1) {
      double* st = a.colstats + (size_t)(g % kSlots) * 2 * 64;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        atomicAdd(&st[wave * 16 + fq * 4 + r], (double)s1[r]);
        atomicAdd(&st[64 + wave * 16 + fq * 4 + r], (double)s2[r]);
      }
    }
  }
}

// dst[i] += sum over s < splits of part[s][i] (n % 4 == 0): block = 64 consecutive elements (16 float4 columns) x 16
// split groups (group j sums splits j, j + 16, ... in order), the groups summed in a fixed order through LDS —
// every thread keeps its loads in flight (the generic split-K reduction walks all splits serially per thread:
// 63 us for 256 partials of 36,864 floats)
__global__ __launch_bounds__(256) void part_reduce_kernel(const float* __restrict__ part, int splits, long long n,
                                                          float* __restrict__ dst) {
  __shared__ float4 red[16][16];
  const int col = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const long long n4 = n >> 2, i4 = (long long)blockIdx.x * 16 + col;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < n4) {
    const float4* p4 = reinterpret_cast<const float4*>(part);
#pragma unroll 4
    for (int s = grp; s < splits; s += 16) {
      const float4 v = p4[(size_t)s * n4 + i4];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  red[grp][col] = acc;
  __syncthreads();
  if (grp == 0 && i4 < n4) {
    float4 t = red[0][col];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      const float4 v = red[j][col];
      t.x += v.x;
      t.y += v.y;
      t.z += v.z;
      t.w += v.w;
    }
    float4* d4 = reinterpret_cast<float4*>(dst);
    float4 d = d4[i4];
    d.x += t.x;
    d.y += t.y;
    d.z += t.z;
    d.w += t.w;
    d4[i4] = d;
  }
}

}  // namespace halo
}  // namespace tde

using namespace tde;

static int halo_lds_bytes(int W, int TR) { return halo::kWBytes + (2 * TR + 4) * ((W + 2) * halo::kPix + 64); }

typedef void (*HaloKern)(halo::Args);
template <int TR, int PB>
static HaloKern halo_kern4(bool acc, bool allv) {
  if (acc) return allv ? halo::conv3x3_kernel<TR, PB, true, true> : halo::conv3x3_kernel<TR, PB, true, false>;
  return allv ? halo::conv3x3_kernel<TR, PB, false, true> : halo::conv3x3_kernel<TR, PB, false, false>;
}
// the instantiated forms: PB = ceil(TR * W / 32) rounded up to 4 or 7; ALLV when the 2 x PB blocks tile
// the TR rows exactly (ResNet-18 stage 1: 4 x 56 = 14 blocks of 16)
static HaloKern halo_kernel(int tr, int pb, bool acc, bool allv) {
  if (pb > 7) return nullptr;
  if (pb > 4) {
    if (tr == 4) return halo_kern4<4, 7>(acc, allv);
    if (tr == 2) return halo_kern4<2, 7>(acc, allv);
    if (tr == 8) return halo_kern4<8, 7>(acc, allv);
    return nullptr;
  }
  if (tr == 2) return halo_kern4<2, 4>(acc, allv);
  if (tr == 4) return halo_kern4<4, 4>(acc, allv);
  if (tr == 8) return halo_kern4<8, 4>(acc, allv);
  return nullptr;
}

// rows per tile: the largest TR in {8, 4, 2} with H % TR == 0, at most 7 pixel blocks per wave
// (TR * W <= 224) and the LDS footprint <= 160 KiB
static int halo_rows(int H, int W) {
  for (int tr : {8, 4, 2})
    if (H % tr == 0 && tr * W <= 224 && halo_lds_bytes(W, tr) <= 160 * 1024) return tr;
  return 0;
}

static long long* g_halo_stamps = nullptr;
// diagnostics: the next launches record per-workgroup phase clocks ([grid][kMaxStamps] s_memrealtime ticks)
TDE_API void tde_halo_stamps(long long* buf) { g_halo_stamps = buf; }

TDE_API int tde_halo_conv_ok(int C, int Co, int H, int W, int B) {
  if (C != halo::kC || Co != halo::kC) return 0;
  if (W % 8 != 0 || W < 8 || H < 2) return 0;
  if ((long long)B * H * W * halo::kPix >= (1LL << 31)) return 0;
  const int tr = halo_rows(H, W);
  return tr > 0 && halo_kernel(tr, (tr * W + 31) / 32, false, false) != nullptr;
}

// y[B,H,W,64] (=|+=) conv3x3_s1_same(x, w); weights element (tap, n, k) at w[tap' * wst + n * wsn + k]
TDE_API int tde_halo_conv3x3(const bf16* x, const bf16* w, long long wst, long long wsn, int flip, bf16* y, int accum,
                             double* colstats, int B, int H, int W, int grid, hipStream_t stream) {
  if (!tde_halo_conv_ok(64, 64, H, W, B)) return -2;
  if (((uintptr_t)x & 15) || ((uintptr_t)w & 15) || ((uintptr_t)y & 7) || (wst % 8) || (wsn % 8)) return -3;
  const int tr = halo_rows(H, W);
  const int lds = halo_lds_bytes(W, tr);
  const int pbn = (tr * W + 31) / 32;
  const int pbk = pbn > 4 ? 7 : 4;
  const HaloKern fn = halo_kernel(tr, pbn, accum != 0, tr * W == 32 * pbk);
  static HaloKern attr_done[16] = {nullptr};
  bool done = false;
  for (int i = 0; i < 16 && attr_done[i]; ++i) done |= attr_done[i] == fn;
  if (!done) {
    if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
      return -4;
    for (int i = 0; i < 16; ++i)
      if (!attr_done[i]) {
        attr_done[i] = fn;
        break;
      }
  }
  const int ntiles = B * (H / tr);
  if (grid <= 0) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    grid = cus;
  }
  if (grid > ntiles) grid = ntiles;
  halo::Args a{x, w, wst, wsn, flip, y, accum, colstats, B, H, W, (int)((long long)B * H * W * halo::kPix),
               g_halo_stamps};
  hipLaunchKernelGGL(fn, dim3(grid), dim3(256), lds, stream, a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// ---- weight gradient (wgrad3x3_kernel)
static int halo_wg_lds(int W, int TR) { return (2 * TR + 4) * (W + 2) * halo::kWgPix + 2 * TR * W * halo::kWgPix; }
// rows per tile: the largest TR in {4, 2} with H % TR == 0, whole 32-pixel k-steps and the LDS <= 160 KiB
static int halo_wg_rows(int H, int W) {
  for (int tr : {4, 2})
    if (H % tr == 0 && (tr * W) % 32 == 0 && halo_wg_lds(W, tr) <= 160 * 1024) return tr;
  return 0;
}
static int halo_wg_grid(int B, int H, int W) {
  static const int env = [] {
    const char* e = getenv("TDE_HALO_WG_GRID");
    return e ? atoi(e) : 0;
  }();
  int grid = env;
  if (grid <= 0) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    grid = cus;
  }
  const int tr = halo_wg_rows(H, W);
  const int ntiles = tr ? B * (H / tr) : 1;
  return grid > ntiles ? ntiles : grid;
}

// MFMA shape of the weight gradient: TDE_HALO_WG_MFMA = 16 | 32 (default 16); tde_halo_wgrad_mfma (tests, A/B).
// The 32x32x16 form measured slower on ResNet-18 stage 1 (30.4 -> 37.1 us per layer, 22.48k -> 22.28k img/s,
// profiles/r6_halo_wgrad/): it needs 10 transposed fragment reads per 9 MFMAs of 16 pixels against 13 per 36
// MFMAs of 32 pixels, and the LDS reads, not the MFMA issue, bound this loop.
static int g_hwg_mf = [] {
  const char* e = getenv("TDE_HALO_WG_MFMA");
  return e && atoi(e) == 32 ? 32 : 16;
}();
TDE_API void tde_halo_wgrad_mfma(int mf) { g_hwg_mf = mf == 32 ? 32 : 16; }

TDE_API int tde_halo_wgrad_ok(int C, int Co, int H, int W, int B) {
  if (C != halo::kC || Co != halo::kC || W % 8 != 0 || W < 8) return 0;
  if ((long long)B * H * W * halo::kWgPix >= (1LL << 31)) return 0;
  return halo_wg_rows(H, W) > 0;
}
// f32 elements of the per-workgroup partials of one launch (the plan's weight-gradient scratch)
TDE_API long long tde_halo_wgrad_scratch_elems(int B, int H, int W) {
  return (long long)halo_wg_grid(B, H, W) * 9 * 64 * 64;
}

// dW[3][3][64][64] (f32, HWIO) += sum over pixels of x (x) dY, 3x3 / stride 1 / SAME; part: scratch of
// tde_halo_wgrad_scratch_elems floats
TDE_API int tde_halo_wgrad3x3(const bf16* x, const bf16* dy, float* dW, float* part, long long part_elems, int B,
                              int H, int W, hipStream_t stream) {
  if (!tde_halo_wgrad_ok(64, 64, H, W, B)) return -2;
  if (((uintptr_t)x & 15) || ((uintptr_t)dy & 15) || ((uintptr_t)dW & 15) || ((uintptr_t)part & 15)) return -3;
  const int tr = halo_wg_rows(H, W);
  const int grid = halo_wg_grid(B, H, W);
  if (part_elems < (long long)grid * 9 * 64 * 64) return -5;
  const int lds = halo_wg_lds(W, tr);
  const int mf = g_hwg_mf;
  void (*fn)(halo::WgArgs) = mf == 32 ? (tr == 4 ? halo::wgrad3x3_kernel<4, 32> : halo::wgrad3x3_kernel<2, 32>)
                                      : (tr == 4 ? halo::wgrad3x3_kernel<4, 16> : halo::wgrad3x3_kernel<2, 16>);
  static void (*attr[4])(halo::WgArgs) = {nullptr, nullptr, nullptr, nullptr};
  bool done = false;
  for (int i = 0; i < 4 && attr[i]; ++i) done |= attr[i] == fn;
  if (!done) {
    if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
      return -4;
    for (int i = 0; i < 4; ++i)
      if (!attr[i]) {
        attr[i] = fn;
        break;
      }
  }
  halo::WgArgs a{x, dy, part, B, H, W, (int)((long long)B * H * W * halo::kWgPix)};
  hipLaunchKernelGGL(fn, dim3(grid), dim3(256), lds, stream, a);
  TDE_LAUNCH_CHECK();
  const long long n = 9LL * 64 * 64;
  halo::part_reduce_kernel<<<(int)((n / 4 + 15) / 16), 256, 0, stream>>>(part, grid, n, dW);
  TDE_LAUNCH_CHECK();
  return 0;
}

// ---- packed-stem weight gradient (stem_wgrad_kernel)
constexpr int kStemTR = 2;
static int stem_wg_lds(int KH, int sh, int Wo) {
  return 2 * ((kStemTR - 1) * sh + KH) * halo::kSxRow + 2 * kStemTR * Wo * halo::kWgPix;
}
// the virtual geometry (C = 8, KWv = 4 taps, stride (sh, 1), valid) with 64 output channels
TDE_API int tde_stem_wgrad_ok(int B, int Hp, int Wv, int Ho, int Wo, int KH, int KWv, int sh, int C, int Co) {
  if (C != 8 || Co != 64 || KWv != 4 || KH < 1 || KH > 8 || sh < 1) return 0;
  if (Wo % 8 || (kStemTR * Wo) % 32 || Ho % kStemTR || Wv != Wo + 3 || Wv > 128 || Hp < (Ho - 1) * sh + KH) return 0;
  if ((long long)B * Hp * Wv * 16 >= (1LL << 31) || (long long)B * Ho * Wo * 128 >= (1LL << 31)) return 0;
  return stem_wg_lds(KH, sh, Wo) <= 160 * 1024;
}
TDE_API long long tde_stem_wgrad_scratch_elems(int B, int Ho, int KH) {
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int ntiles = B * (Ho / kStemTR);
  const int grid = cus < ntiles ? cus : ntiles;
  return (long long)grid * 2 * KH * 16 * 64;
}
// dWv[KH][4][8][64] (f32) += the packed stem's weight gradient; part: tde_stem_wgrad_scratch_elems floats
TDE_API int tde_stem_wgrad(const bf16* xp, const bf16* dy, float* dWv, float* part, long long part_elems, int B, int Hp,
                           int Wv, int Ho, int Wo, int KH, int sh, hipStream_t stream) {
  if (!tde_stem_wgrad_ok(B, Hp, Wv, Ho, Wo, KH, 4, sh, 8, 64)) return -2;
  if (((uintptr_t)xp & 15) || ((uintptr_t)dy & 15) || ((uintptr_t)dWv & 15) || ((uintptr_t)part & 15)) return -3;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int ntiles = B * (Ho / kStemTR);
  const int grid = cus < ntiles ? cus : ntiles;
  const long long n = 2LL * KH * 16 * 64;
  if (part_elems < (long long)grid * n) return -5;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)halo::stem_wgrad_kernel<kStemTR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return -4;
    attr = true;
  }
  halo::StemWgArgs a{xp, dy, part, B, Hp, Wv, Ho, Wo, KH, sh, (int)((long long)B * Hp * Wv * 16),
                     (int)((long long)B * Ho * Wo * 128)};
  hipLaunchKernelGGL(halo::stem_wgrad_kernel<kStemTR>, dim3(grid), dim3(256), stem_wg_lds(KH, sh, Wo), stream, a);
  TDE_LAUNCH_CHECK();
  halo::part_reduce_kernel<<<(int)((n / 4 + 15) / 16), 256, 0, stream>>>(part, grid, n, dWv);
  TDE_LAUNCH_CHECK();
  return 0;
}

// ---- packed-stem forward (stem_fwd_kernel): TR output rows per tile (TDE_STEM_FWD_TR = 2 (default), 4 or 8)
static int stem_fwd_tr() {
  static const int tr = [] {
    const char* e = getenv("TDE_STEM_FWD_TR");
    const int v = e ? atoi(e) : 2;   // 43.5 / 45.0 / 86.6 us per stem at 2 / 4 / 8 (profiles/r6_stem_fwd/)
    return v == 4 || v == 8 ? v : 2;
  }();
  return tr;
}
static int stem_fwd_lds(int KH, int sh, int Wo) {
  (void)Wo;
  return 2 * ((stem_fwd_tr() - 1) * sh + KH) * halo::kSxRow;
}
TDE_API int tde_stem_fwd_ok(int B, int Hp, int Wv, int Ho, int Wo, int KH, int KWv, int sh, int C, int Co) {
  if (C != 8 || Co != 64 || KWv != 4 || KH < 1 || KH > 8 || sh < 1) return 0;
  if (Wo % 16 || Ho % stem_fwd_tr() || Wv != Wo + 3 || Wv > 128 || Hp < (Ho - 1) * sh + KH) return 0;
  if ((long long)B * Hp * Wv * 16 >= (1LL << 31)) return 0;
  return stem_fwd_lds(KH, sh, Wo) <= 160 * 1024;
}
// y [B][Ho][Wo][64] bf16 = the packed stem conv of xp with wv [64][KH * 32]; colstats (nullable) += its BN sums
TDE_API int tde_stem_fwd(const bf16* xp, const bf16* wv, bf16* y, double* colstats, int B, int Hp, int Wv, int Ho, int Wo,
                         int KH, int sh, hipStream_t stream) {
  if (!tde_stem_fwd_ok(B, Hp, Wv, Ho, Wo, KH, 4, sh, 8, 64)) return -2;
  if (((uintptr_t)xp & 15) || ((uintptr_t)wv & 15) || ((uintptr_t)y & 15) || ((uintptr_t)colstats & 7)) return -3;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  static const int per_cu = [] {
    const char* e = getenv("TDE_STEM_FWD_GRID");
    return e && atoi(e) > 0 ? atoi(e) : 0;
  }();
  const int ntiles = B * (Ho / stem_fwd_tr());
  // what fits a CU's LDS at once, at most 3 (2 / 3 / 4 per CU: 49.7 / 41.7 / 45.0 us, profiles/r6_stem_fwd/grid.txt)
  const int fit = (160 * 1024) / stem_fwd_lds(KH, sh, Wo);
  const int per_cu_ = per_cu ? per_cu : (fit < 3 ? fit : 3);
  const int grid = cus * per_cu_ < ntiles ? cus * per_cu_ : ntiles;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)halo::stem_fwd_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess ||
        hipFuncSetAttribute((const void*)halo::stem_fwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess ||
        hipFuncSetAttribute((const void*)halo::stem_fwd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return -4;
    attr = true;
  }
  halo::StemFwdArgs a{xp, wv, y, colstats, B, Hp, Wv, Ho, Wo, KH, sh, (int)((long long)B * Hp * Wv * 16)};
  const int lds = stem_fwd_lds(KH, sh, Wo);
  if (stem_fwd_tr() == 8) hipLaunchKernelGGL(halo::stem_fwd_kernel<8>, dim3(grid), dim3(256), lds, stream, a);
  else if (stem_fwd_tr() == 4) hipLaunchKernelGGL(halo::stem_fwd_kernel<4>, dim3(grid), dim3(256), lds, stream, a);
  else hipLaunchKernelGGL(halo::stem_fwd_kernel<2>, dim3(grid), dim3(256), lds, stream, a);
  TDE_LAUNCH_CHECK();
  return 0;
}

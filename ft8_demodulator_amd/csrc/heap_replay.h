// heap_replay.h -- the reference candidate heap rebuilt in the registers of one wave.
//
// ft8_find_candidates (ft8_decode.py:113-140) keeps its candidates in a Python heapq of
// (-score, candidate) tuples; when two selected scores are exactly equal, the order the reference
// returns them in (sorted(..., key=-score) over the heap ARRAY, ft8_decode.py:139) depends on
// where the heap left them.  The final array is the heap of the first N passing candidates --
// N heappushes in scan order (heapq._siftdown) -- with its root replaced by the last record, a
// later strict new maximum (heapreplace = _siftup along the min-child path, then _siftdown of the
// record, which lands back at the root).
//
// Layout: heap position P (1-based) sits in register P >> 6, lane P & 63, as the pair
// (monotone(-score), scan index) whose unsigned lexicographic order is the reference's tuple order
// (scan indices are distinct, so no two tuples are equal).  The parents of positions in register
// k live in register k >> 1, so every register index is a compile-time constant; lanes are
// addressed with readlane / writelane on wave-uniform indices and each push stops at its first
// non-passing parent, exactly like _siftdown.  Positions 1..511 (kReplayRegs registers).
//
// A comparison between two tuples whose scores are equal is where the reference would go on to
// compare FT8Candidate objects (which define no ordering -> TypeError); the functions return 1
// when such a comparison happens.
#pragma once
#include <hip/hip_runtime.h>

namespace ft8 {

constexpr int kReplayRegs = 8;
constexpr int kReplayMax = 64 * kReplayRegs - 1;  // largest heap the register replay holds

// -s as a float with -0 folded onto +0, mapped to an unsigned key of the same order
__device__ inline unsigned mono_neg(float s) {
  const unsigned u = __float_as_uint(0.0f - s);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline unsigned rdl(unsigned v, unsigned l) {
  return (unsigned)__builtin_amdgcn_readlane((int)v, (int)l);
}
// the writelane intrinsic (the compiler routes its lane select through M0)
extern "C" __device__ int ft8_writelane(int x, int lane, int v) __asm("llvm.amdgcn.writelane");
__device__ inline void wrl(unsigned& h, unsigned& l, unsigned xh, unsigned xl, unsigned n) {
  h = (unsigned)ft8_writelane((int)xh, (int)n, (int)h);
  l = (unsigned)ft8_writelane((int)xl, (int)n, (int)l);
}
__device__ inline bool tuple_lt(unsigned ah, unsigned al, unsigned bh, unsigned bl) {
  return ah < bh || (ah == bh && al < bl);
}

// position P (1-based, uniform) of the register heap
__device__ inline void heap_get(const unsigned (&hh)[kReplayRegs], const unsigned (&hl)[kReplayRegs], unsigned P,
                                unsigned& h, unsigned& l) {
  const unsigned k = P >> 6, n = P & 63;
  h = 0;
  l = 0;
#pragma unroll
  for (int j = 0; j < kReplayRegs; ++j)
    if (k == (unsigned)j) {
      h = rdl(hh[j], n);
      l = rdl(hl[j], n);
    }
}
__device__ inline void heap_set(unsigned (&hh)[kReplayRegs], unsigned (&hl)[kReplayRegs], unsigned P, unsigned h,
                                unsigned l) {
  const unsigned k = P >> 6, n = P & 63;
#pragma unroll
  for (int j = 0; j < kReplayRegs; ++j)
    if (k == (unsigned)j) wrl(hh[j], hl[j], h, l, n);
}

// Items in push order: lane l of register k gets push n = 64k + l - 1 (heap position 64k + l),
// scan index push[n], score psc[n].  nsel <= kReplayMax.
template <typename IdxPtr>
__device__ inline void heap_load(const float* psc, IdxPtr push, int nsel, unsigned (&hh)[kReplayRegs],
                                 unsigned (&hl)[kReplayRegs]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < kReplayRegs; ++k) {
    const int n = 64 * k + lane - 1;
    unsigned h = 0, l = 0;
    if (n >= 0 && n < nsel) {
      const int idx = push[n];
      h = mono_neg(psc[n]);
      l = (unsigned)idx;
    }
    hh[k] = h;
    hl[k] = l;
  }
}

// The N heappushes (ft8_decode.py:128-133 -> heapq._siftdown).  Returns the tie flag.
__device__ inline int heap_pushes(int nsel_in, unsigned (&hh)[kReplayRegs], unsigned (&hl)[kReplayRegs]) {
  const int nsel = __builtin_amdgcn_readfirstlane(nsel_in);
  int tie = 0;
#pragma unroll
  for (int k = 0; k < kReplayRegs; ++k) {
    if (64 * k > nsel) break;
    const int lend = min(64, nsel + 1 - 64 * k);
    for (int l = (k == 0 ? 2 : 0); l < lend; ++l) {
      // push of the item already sitting at position P = 64k + l (positions 1..P-1 form the heap)
      const unsigned nh = rdl(hh[k], l), nl = rdl(hl[k], l);
      unsigned P = 64u * k + l;
      bool climbing = true;
#pragma unroll
      for (int j = 1; j <= 3; ++j) {  // parents outside register 0
        const int rc = k >> (j - 1), rp = k >> j;
        if (rc == 0) break;
        if (climbing) {
          const unsigned pp = P >> 1;
          const unsigned ph = rdl(hh[rp], pp & 63), pl = rdl(hl[rp], pp & 63);
          if (ph == nh) tie = 1;
          if (tuple_lt(nh, nl, ph, pl)) {
            wrl(hh[rc], hl[rc], ph, pl, P & 63);
            P = pp;
          } else {
            if (j > 1) wrl(hh[rc], hl[rc], nh, nl, P & 63);
            climbing = false;
          }
        }
      }
      if (climbing) {
        bool moved = k > 0;
        while (P > 1) {
          const unsigned pp = P >> 1;
          const unsigned ph = rdl(hh[0], pp), pl = rdl(hl[0], pp);
          if (ph == nh) tie = 1;
          if (!tuple_lt(nh, nl, ph, pl)) break;
          wrl(hh[0], hl[0], ph, pl, P);
          P = pp;
          moved = true;
        }
        if (moved) wrl(hh[0], hl[0], nh, nl, P);
      }
    }
  }
  return tie;
}

// The records' heapreplace (ft8_decode.py:134-137): _siftup compares siblings along the min-child
// path (the same path for every record, since it ends with the record back at the root), then the
// root holds the last record.  Returns the tie flag of those sibling comparisons.
__device__ inline int heap_record(int nsel_in, unsigned (&hh)[kReplayRegs], unsigned (&hl)[kReplayRegs], unsigned rh,
                                  unsigned rl) {
  const unsigned nsel = (unsigned)__builtin_amdgcn_readfirstlane(nsel_in);
  int tie = 0;
  unsigned C = 2;
  while (C <= nsel) {
    const unsigned R = C + 1;
    if (R <= nsel) {
      unsigned ch, cl, sh, sl;
      heap_get(hh, hl, C, ch, cl);
      heap_get(hh, hl, R, sh, sl);
      if (ch == sh) tie = 1;
      if (!tuple_lt(ch, cl, sh, sl)) C = R;
    }
    C <<= 1;
  }
  wrl(hh[0], hl[0], rh, rl, 1);
  return tie;
}

}  // namespace ft8

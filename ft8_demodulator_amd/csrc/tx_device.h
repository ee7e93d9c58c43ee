// tx_device.h -- the FT8 transmit chain as device functions (gfx950), shared by tx.hip (waveform
// synthesis) and subtract.hip (re-modulation of decoded messages for subtract-and-redecode).
//
//   payload (77 bits) -> a91 = payload | CRC-14      ft8_generator/crc.py:25-47 crc_generator
//   a91 -> 174-bit codeword (83 parity bits)          ft8_generator/ldpc.py:104-131 ldpc_generator
//   codeword -> 58 Gray-mapped 3-bit symbols          ft8_generator/encoder.py:15-37
//   + Costas-7 at 0/36/72 -> 79 tones                 ft8_generator/encoder.py:39-64
//   tones -> GFSK phase                               ft8_generator/modulator.py:27-74
//
// The GFSK phase is evaluated in closed form instead of the reference's sequential
// phi = fmod(phi + dphi[i], 2 pi) loop (modulator.py:64-68), so every sample is independent:
//   freq_seq[m] = 6.25 * sum_{j=-1}^{79} e_j * p(m - j*nsps)           (modulator.py:41-48)
// with e_{-1} = tone_0, e_79 = tone_78 (the extension pulses of modulator.py:46-48) and p the
// Gaussian frequency pulse of length 3*nsps (gauss_window_generator, modulator.py:20-25).  With
// P(x) = sum_{y<x} p(y) (0 for x <= 0, P(3 nsps) beyond) the running phase of sample n is
//   phi(n) = 2 pi / fs * (f0 * n + 6.25 * (G(n + off) - G(off))),  G(u) = sum_j e_j P(u - j nsps)
// where only three pulses are partial at any u.  off = 0 reproduces the reference modulator
// (which reads freq_seq without the one-symbol offset, so its symbols start one symbol late);
// off = nsps is the protocol timing (symbol i occupies samples [i nsps, (i+1) nsps)).
#pragma once
#include "ft8_internal.h"

namespace ft8 {
namespace tx {

constexpr int kSymbols = 79;
constexpr int kExt = 81;  // e_{-1} .. e_79

namespace {
__constant__ __attribute__((aligned(16))) uint8_t kGenRowsTx[FT8_LDPC_M * 12] = FT8_GEN_ROWS_INIT;
__constant__ uint8_t kCostasTx[7] = {3, 1, 4, 0, 6, 5, 2};  // encoder.py:11
__constant__ uint8_t kGrayTx[8] = {0, 1, 3, 2, 5, 6, 4, 7};   // encoder.py:10
}  // namespace

__device__ __forceinline__ uint64_t be64(const uint8_t* b, int n) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) v = (v << 8) | (i < n ? (uint64_t)b[i] : 0ull);
  return v;
}

// CRC-14 (poly 0x2757, MSB first, init 0) of the first nbits of the big-endian bit string
// (w0, w1) -- crc.py:9-22 calc_crc, bit-serial form of its byte loop
__device__ __forceinline__ unsigned crc14_words(uint64_t w0, uint64_t w1, int nbits) {
  unsigned rem = 0;
  for (int i = 0; i < nbits; ++i) {
    const unsigned b = (unsigned)(((i < 64 ? w0 : w1) >> (63 - (i & 63))) & 1ull);
    rem ^= b << 13;
    rem = (rem & 0x2000u) ? ((rem << 1) ^ 0x2757u) : (rem << 1);
  }
  return rem & 0x3FFFu;
}

// msg -> a91[12], codeword[22], tones[79] (each output nullable).  msg_bytes 10: msg is a payload
// and a91 = crc_generator(payload); 12: msg is an a91 taken as given (ldpc_generator's input, whose
// 12 bytes are copied into the codeword before the parity bits are OR-ed in, ldpc.py:106-109).
__device__ inline void encode(const uint8_t* msg, int msg_bytes, uint8_t* a91, uint8_t* cw, uint8_t* tones) {
  uint64_t m0, m1;
  if (msg_bytes == 12) {
    m0 = be64(msg, 8);
    m1 = be64(msg + 8, 4);
  } else {
    uint8_t p[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) p[i] = msg[i];
    p[9] &= 0xF8;                                      // crc.py:35
    m0 = be64(p, 8);
    const uint64_t m1p = be64(p + 8, 2);               // bytes 8, 9 (10, 11 zero: crc.py:36-37)
    const unsigned crc = crc14_words(m0, m1p, 82);     // 96 - 14 bits (crc.py:40)
    // a91 bytes 8..11: p[8], p[9] | crc >> 11, crc >> 3, crc << 5 (crc.py:43-45)
    m1 = m1p | ((uint64_t)(crc >> 11) << 48) | ((uint64_t)((crc >> 3) & 0xFF) << 40) |
         ((uint64_t)((crc << 5) & 0xE0) << 32);
  }
  // parity bits: row i of G against the 91 message bits (ldpc.py:117-129)
  uint64_t par0 = 0, par1 = 0;  // parity bit i at position i of (par0: 0..63, par1: 64..82), MSB first
  for (int i = 0; i < FT8_LDPC_M; ++i) {
    const uint8_t* g = kGenRowsTx + i * 12;
    const uint64_t g0 = be64(g, 8), g1 = be64(g + 8, 4);
    const unsigned bit = (unsigned)(__popcll(g0 & m0) + __popcll(g1 & m1)) & 1u;
    if (i < 64) par0 |= (uint64_t)bit << (63 - i);
    else par1 |= (uint64_t)bit << (63 - (i - 64));
  }
  // codeword bit string: bits 0..90 message, 91..173 parity
  const uint64_t c0 = m0;
  const uint64_t c1 = (m1 & 0xFFFFFFFF00000000ull) | (par0 >> 27);  // a91 byte 11 | first parity bits
  const uint64_t c2 = (par0 << 37) | (par1 >> 27);
  if (a91) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a91[i] = (uint8_t)(m0 >> (56 - 8 * i));
#pragma unroll
    for (int i = 0; i < 4; ++i) a91[8 + i] = (uint8_t)(m1 >> (56 - 8 * i));
  }
  if (cw) {
#pragma unroll
    for (int i = 0; i < 8; ++i) cw[i] = (uint8_t)(c0 >> (56 - 8 * i));
#pragma unroll
    for (int i = 0; i < 8; ++i) cw[8 + i] = (uint8_t)(c1 >> (56 - 8 * i));
#pragma unroll
    for (int i = 0; i < 6; ++i) cw[16 + i] = (uint8_t)(c2 >> (56 - 8 * i));
  }
  if (tones) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      tones[k] = kCostasTx[k];
      tones[36 + k] = kCostasTx[k];
      tones[72 + k] = kCostasTx[k];
    }
#pragma unroll
    for (int s = 0; s < 58; ++s) {
      unsigned v = 0;
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const int i = 3 * s + b;
        const uint64_t w = i < 64 ? c0 : (i < 128 ? c1 : c2);
        v = (v << 1) | (unsigned)((w >> (63 - (i & 63))) & 1ull);
      }
      tones[s < 29 ? 7 + s : 14 + s] = kGrayTx[v];
    }
  }
}

// One wave encodes one payload into tones[79] (LDS or global): the 83 parity rows are spread over
// the lanes (rows l and l + 64) and gathered with two ballots, the 58 data symbols one per lane.
// Same bits as encode(); used where a single message must be encoded with low latency.
__device__ inline void encode_tones_wave(const uint8_t* payload, int lane, uint8_t* tones) {
  uint8_t p[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) p[i] = payload[i];
  p[9] &= 0xF8;
  const uint64_t m0 = be64(p, 8);
  const uint64_t m1p = be64(p + 8, 2);
  const unsigned crc = crc14_words(m0, m1p, 82);
  const uint64_t m1 = m1p | ((uint64_t)(crc >> 11) << 48) | ((uint64_t)((crc >> 3) & 0xFF) << 40) |
                      ((uint64_t)((crc << 5) & 0xE0) << 32);
  auto row_bit = [&](int row) -> bool {
    const uint32_t* g = reinterpret_cast<const uint32_t*>(kGenRowsTx) + row * 3;
    const uint64_t g0 = ((uint64_t)__builtin_bswap32(g[0]) << 32) | __builtin_bswap32(g[1]);
    const uint64_t g1 = (uint64_t)__builtin_bswap32(g[2]) << 32;
    return ((__popcll(g0 & m0) + __popcll(g1 & m1)) & 1) != 0;
  };
  const bool ba = row_bit(lane);
  const bool bb = lane + 64 < FT8_LDPC_M ? row_bit(lane + 64) : false;
  const uint64_t par0 = __builtin_bitreverse64(__ballot(ba));  // parity i at bit 63 - i
  const uint64_t par1 = __builtin_bitreverse64(__ballot(bb));
  const uint64_t c0 = m0;
  const uint64_t c1 = (m1 & 0xFFFFFFFF00000000ull) | (par0 >> 27);
  const uint64_t c2 = (par0 << 37) | (par1 >> 27);
  if (lane < 7) {
    tones[lane] = kCostasTx[lane];
    tones[36 + lane] = kCostasTx[lane];
    tones[72 + lane] = kCostasTx[lane];
  }
  if (lane < 58) {
    unsigned v = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int i = 3 * lane + b;
      const uint64_t w = i < 64 ? c0 : (i < 128 ? c1 : c2);
      v = (v << 1) | (unsigned)((w >> (63 - (i & 63))) & 1ull);
    }
    tones[lane < 29 ? 7 + lane : 14 + lane] = kGrayTx[v];
  }
}

// G(u) = sum_j e_j P(u - j nsps), E[0..80] = e_{-1..79}, PS[k] = sum_{i<k} E[i] (k = 0..81),
// P[0..3 nsps] the cumulative pulse.  Exact in double when P is double.
template <typename PT, typename AT>
__device__ __forceinline__ AT gfsk_G(const int* E, const int* PS, const PT* P, int nsps, int u) {
  const int q = u / nsps, r = u - q * nsps;                   // u >= 0
  const int full = min(max(q - 1, 0), kExt);                  // pulses j <= q - 3 are complete
  AT s = (AT)PS[full] * (AT)P[3 * nsps];
  if (q - 1 >= 0 && q - 1 < kExt) s += (AT)E[q - 1] * (AT)P[r + 2 * nsps];  // j = q - 2
  if (q < kExt) s += (AT)E[q] * (AT)P[r + nsps];                              // j = q - 1
  if (q + 1 < kExt) s += (AT)E[q + 1] * (AT)P[r];                             // j = q
  return s;
}

// amplitude ramp of modulator.py:70-73 at sample n of a 79*nsps waveform.  style 1 reproduces the
// reference exactly (its trailing ramp rises to 1 at the last sample); style 0 ramps down.
template <typename T>
__device__ __forceinline__ T gfsk_ramp(int n, int L, int nsps, int style) {
  const int nramp = nsps / 8;
  if (n < nramp) return (T)0.5 * ((T)1 - cos((T)(8.0 * M_PI) * (T)n / (T)nsps));
  const int i = L - 1 - n;
  if (i < nramp) {
    const T c = cos((T)(8.0 * M_PI) * (T)i / (T)nsps);
    return style == 1 ? (T)0.5 * ((T)1 + c) : (T)0.5 * ((T)1 - c);
  }
  return (T)1;
}

}  // namespace tx
}  // namespace ft8

/* decode_wav.c -- libft8hip.so from plain C: decode one 16-bit PCM WAV slot the way the reference's
 * CLI does (src/tests/demodulator/from_wave.py: read_wave_file, then decode_ft8_message with its
 * keyword defaults, ft8_decode.py:288-296), with nothing but the C-ABI of include/ft8hip.h and the
 * HIP runtime.  One line per decode:
 *
 *   payload_hex crc_calculated ldpc_errors crc_extracted time_sec freq_hz score
 *
 * time_sec = abs_time / fs and freq_hz = (abs_freq / bins_per_tone) * 6.25, as the reference
 * computes them (ft8_decode.py:383-391); the score is the float32 sync score widened to double.
 *
 *   make -C examples            (gcc, links ../ft8_demodulator_amd/lib/libft8hip.so)
 *   examples/decode_wav FILE.wav [-k max_candidates] [-s min_score] [-i max_iterations]
 *                                [-b bins_per_tone] [-p steps_per_symbol]
 *
 * tests/test_gpu_binding.py runs it on the reference's bundled recording and the synthetic WAVs
 * against the reference's golden decodes. */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ft8hip.h"

static int fail(const char* what) {
  fprintf(stderr, "decode_wav: %s\n", what);
  return 1;
}

static uint32_t le32(const unsigned char* p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }
static uint16_t le16(const unsigned char* p) { return (uint16_t)(p[0] | p[1] << 8); }

/* read_wave_file (from_wave.py:24-69): 16-bit PCM only, the first channel of a multi-channel file.
 * Returns the channel-0 samples as int16 (the library applies the reference's x / 32767 on the
 * device, FT8_I16). */
static int16_t* read_wav(const char* path, int64_t* n_out, int* fs_out) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long size = ftell(f);
  fseek(f, 0, SEEK_SET);
  unsigned char* b = (unsigned char*)malloc((size_t)size);
  if (!b || fread(b, 1, (size_t)size, f) != (size_t)size) {
    fclose(f);
    free(b);
    return NULL;
  }
  fclose(f);
  int16_t* out = NULL;
  int channels = 0, bits = 0, fmt = 0, fs = 0;
  if (size < 12 || memcmp(b, "RIFF", 4) || memcmp(b + 8, "WAVE", 4)) goto done;
  for (long pos = 12; pos + 8 <= size;) {
    const uint32_t len = le32(b + pos + 4);
    const unsigned char* body = b + pos + 8;
    if (pos + 8 + (long)len > size) break;
    if (!memcmp(b + pos, "fmt ", 4) && len >= 16) {
      fmt = le16(body);
      channels = le16(body + 2);
      fs = (int)le32(body + 4);
      bits = le16(body + 14);
    } else if (!memcmp(b + pos, "data", 4)) {
      if (fmt != 1 || bits != 16 || channels < 1) break;  /* the reference reads 16-bit PCM */
      const int64_t frames = (int64_t)len / (2 * channels);
      out = (int16_t*)malloc((size_t)(frames > 0 ? frames : 1) * sizeof(int16_t));
      if (!out) break;
      for (int64_t i = 0; i < frames; ++i) out[i] = (int16_t)le16(body + 2 * channels * i);
      *n_out = frames;
      *fs_out = fs;
      break;
    }
    pos += 8 + (long)len + (len & 1);
  }
done:
  free(b);
  return out;
}

int main(int argc, char** argv) {
  if (argc < 2) return fail("usage: decode_wav FILE.wav [-k K] [-s min_score] [-i iterations] [-b bpt] [-p sps]");
  int K = 20, iters = 20, bpt = 2, sps = 2;  /* decode_ft8_message's defaults */
  double min_score = 10.0;
  for (int a = 2; a + 1 < argc; a += 2) {
    if (!strcmp(argv[a], "-k")) K = atoi(argv[a + 1]);
    else if (!strcmp(argv[a], "-s")) min_score = atof(argv[a + 1]);
    else if (!strcmp(argv[a], "-i")) iters = atoi(argv[a + 1]);
    else if (!strcmp(argv[a], "-b")) bpt = atoi(argv[a + 1]);
    else if (!strcmp(argv[a], "-p")) sps = atoi(argv[a + 1]);
    else return fail("unknown option");
  }
  int64_t n = 0;
  int fs = 0;
  int16_t* x = read_wav(argv[1], &n, &fs);
  if (!x) return fail("cannot read a 16-bit PCM WAV file");
  if (ft8_abi_version() != 2) return fail("libft8hip.so is not ABI 2");

  /* the STFT geometry (spectrogram_analyse.py:31-43) and the reference's f >= 0 mask: natural bins
   * [0, (nfft + 1) / 2); every frame */
  int32_t nperseg = 0, hop = 0, nfft = 0, frames = 0;
  if (ft8_geometry_hz((double)fs, bpt, sps, n, &nperseg, &hop, &nfft, &frames) != FT8_OK) return fail("bad geometry");
  ft8_params p;
  memset(&p, 0, sizeof p);
  p.sample_rate = fs;
  p.sample_rate_hz = (double)fs;
  p.bins_per_tone = bpt;
  p.steps_per_symbol = sps;
  p.max_candidates = K;
  p.max_iterations = iters;
  p.min_score = min_score;
  p.min_score_f64 = 0;  /* a Python number threshold: compared in the waterfall's float32 */
  p.f_lo = 0;
  p.f_hi = (nfft + 1) / 2;
  p.t_lo = 0;
  p.t_hi = frames;

  ft8_ctx* ctx = NULL;
  if (ft8_create(0, &ctx) != FT8_OK) return fail("ft8_create failed (no GPU?)");
  void* d_x = NULL;
  ft8_result* d_out = NULL;
  int32_t* d_count = NULL;
  const int cap = K > 0 ? K : 1;
  if (hipMalloc(&d_x, (size_t)(n > 0 ? n : 1) * sizeof(int16_t)) != hipSuccess ||
      hipMalloc((void**)&d_out, (size_t)cap * sizeof(ft8_result)) != hipSuccess ||
      hipMalloc((void**)&d_count, sizeof(int32_t)) != hipSuccess)
    return fail("hipMalloc failed");
  if (n > 0 && hipMemcpy(d_x, x, (size_t)n * sizeof(int16_t), hipMemcpyHostToDevice) != hipSuccess)
    return fail("upload failed");
  int rc = FT8_OK;
  int32_t count = 0;
  if (frames > 0) {
    rc = ft8_decode_batch(ctx, d_x, FT8_I16, n, 1, n, &p, d_out, d_count, cap, NULL);
    if (rc != FT8_OK) {
      fprintf(stderr, "decode_wav: ft8_decode_batch: %s\n", ft8_last_error(ctx));
      return 1;
    }
    if (hipMemcpy(&count, d_count, sizeof count, hipMemcpyDeviceToHost) != hipSuccess) return fail("download failed");
  }  /* else: shorter than one window -- the reference's empty spectrogram, no decodes */
  if (count > cap) count = cap;
  ft8_result* r = (ft8_result*)calloc((size_t)cap, sizeof(ft8_result));
  if (count > 0 && hipMemcpy(r, d_out, (size_t)count * sizeof(ft8_result), hipMemcpyDeviceToHost) != hipSuccess)
    return fail("download failed");
  for (int i = 0; i < count; ++i) {
    char hex[21];
    for (int j = 0; j < 10; ++j) sprintf(hex + 2 * j, "%02x", r[i].payload[j]);
    printf("%s %u %d %u %.17g %.17g %.9g\n", hex, r[i].crc_calculated, r[i].ldpc_errors, r[i].crc_extracted,
           (double)r[i].abs_time / (double)fs, ((double)r[i].abs_freq / (double)bpt) * 6.25, r[i].score);
  }
  free(r);
  free(x);
  hipFree(d_x);
  hipFree(d_out);
  hipFree(d_count);
  ft8_destroy(ctx);
  return 0;
}

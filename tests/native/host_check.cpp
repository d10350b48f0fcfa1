// Host sanitizer check (CPU): the engine's host-side code -- the weight packing of
// mmpfn_finalize_weights (weight_pack.h) and the row hash mmpfn_siphash24_rows (host.cpp) --
// built with g++ -fsanitize=address,undefined by tests/test_host_sanitize.py, run on the model's
// real shapes, its outputs written as raw little-endian arrays into the directory argv[1] for the
// test to compare against independent numpy / torch restatements.
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/mmpfn_hip.h"
#include "weight_pack.h"

using namespace mmpfn;

template <typename T>
static bool dump(const std::string& dir, const char* name, const std::vector<T>& v) {
  FILE* f = std::fopen((dir + "/" + name).c_str(), "wb");
  if (!f) return false;
  const bool ok = std::fwrite(v.data(), sizeof(T), v.size(), f) == v.size();
  return std::fclose(f) == 0 && ok;
}

static std::vector<float> iota_f(size_t n) {  // exact in fp32 below 2^24
  std::vector<float> v(n);
  for (size_t i = 0; i < n; ++i) v[i] = (float)i;
  return v;
}

int main(int argc, char** argv) {
  if (argc != 2) return 2;
  const std::string dir = argv[1];
  const int E = 192, H = 6, Fh = 768;
  bool ok = true;

  // bf16 rounding of every fp32 class: the test compares with torch's conversion
  std::vector<uint32_t> bits = {0x00000000u, 0x80000000u, 0x3f800000u, 0x3f808000u, 0x3f818000u, 0x3f80ffffu,
                                0x7f7fffffu, 0x7f800000u, 0xff800000u, 0x00000001u, 0x007fffffu, 0x80000001u,
                                0x7fc00000u, 0x7f800001u, 0xffc00001u, 0x7f7f8000u, 0x33800000u, 0xc2f6e979u};
  for (uint32_t i = 0; i < 4096; ++i) bits.push_back(i * 0x000fffffu + 0x3c000000u * (i & 1));
  std::vector<float> fin(bits.size());
  std::vector<uint16_t> fout(bits.size());
  for (size_t i = 0; i < bits.size(); ++i) {
    std::memcpy(&fin[i], &bits[i], 4);
    fout[i] = f2bf(fin[i]);
  }
  ok &= dump(dir, "f2bf_in.bin", bits) && dump(dir, "f2bf_out.bin", fout);

  {  // fp16 rounding (PREC_F16 weights): every class, subnormals, overflow
    std::vector<uint16_t> hout(bits.size());
    for (size_t i = 0; i < bits.size(); ++i) hout[i] = f2h(fin[i]);
    ok &= dump(dir, "f2h_out.bin", hout);
  }
  ok &= dump(dir, "transpose_out.bin", transpose_out(iota_f((size_t)E * E), E, E));
  ok &= dump(dir, "rows_f16.bin", permute_rows_f16(iota_f((size_t)E * Fh), E, Fh));
  ok &= dump(dir, "mlp1.bin", pack_mlp1_perm(iota_f((size_t)Fh * E), E, Fh));
  ok &= dump(dir, "mlp2.bin", pack_mlp2_perm(iota_f((size_t)E * Fh), E, Fh));
  {
    std::vector<float> qkv = iota_f((size_t)3 * H * 32 * E), wout = iota_f((size_t)E * H * 32);
    for (float& x : wout) x = -x;  // out-projection values distinct from the QKV ones
    ok &= dump(dir, "feat_rows.bin", pack_feat_rows(qkv, wout, H, E));
    ok &= dump(dir, "feat_rows_f16.bin", pack_feat_rows(qkv, wout, H, E, true));
  }
  {
    const int N = 576, K = E;
    std::vector<float> W((size_t)N * K), c(N), g(K), b(K);
    for (int n = 0; n < N; ++n) {
      c[n] = n / 32.0f;
      for (int k = 0; k < K; ++k) W[(size_t)n * K + k] = ((n * 7 + k * 3) % 17 - 8) / 8.0f;
    }
    for (int k = 0; k < K; ++k) g[k] = 1.0f + k / 256.0f, b[k] = k / 1024.0f - 0.1f;
    fold_ln(W, c, g.data(), b.data(), N, K);
    ok &= dump(dir, "fold_W.bin", W) && dump(dir, "fold_c.bin", c);
  }
  {
    // every tail length of the 8-byte blocks, and the empty row
    std::vector<int64_t> out;
    for (int rb : {0, 1, 7, 8, 9, 15, 16, 17, 31, 33, 100, 768}) {
      const int n = 5;
      std::vector<unsigned char> rows((size_t)n * rb + 1);  // +1: no zero-size allocation
      for (size_t i = 0; i < rows.size(); ++i) rows[i] = (unsigned char)(i * 31 + 7 + rb);
      std::vector<int64_t> h(n);
      if (mmpfn_siphash24_rows(rows.data(), n, rb, h.data()) != MMPFN_OK) ok = false;
      out.insert(out.end(), h.begin(), h.end());
    }
    ok &= dump(dir, "siphash.bin", out);
  }
  std::printf(ok ? "host_check ok\n" : "host_check FAILED\n");
  return ok ? 0 : 1;
}

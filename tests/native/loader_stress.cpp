// Host-side stress driver for native/runtime/loader.cpp, built by tests/native/test_loader_sanitizers.py
// with -fsanitize=address,undefined (and separately -fsanitize=thread): many asynchronous jobs on
// every slot, random row sets, results checked row by row, then destroy with jobs in flight.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

extern "C" {
int rkl_create(void** out, int ntensors, const void* const* bases, const int64_t* row_bytes, int64_t nrows,
               int nthreads, int nslots);
int rkl_submit(void* loader, int slot, const int64_t* idx, int64_t n, void* const* dsts);
int rkl_wait(void* loader, int slot);
int rkl_destroy(void* loader);
}

int main() {
  const int64_t nrows = 3000;
  const int64_t rb[2] = {3136, 8};  // an MNIST image row (f32 28x28) and a label row (int64)
  std::vector<std::vector<unsigned char>> data(2);
  for (int t = 0; t < 2; ++t) {
    data[t].resize(nrows * rb[t]);
    for (int64_t i = 0; i < nrows * rb[t]; ++i) data[t][i] = (unsigned char)((i * 131 + t * 7) & 0xff);
  }
  const void* bases[2] = {data[0].data(), data[1].data()};
  void* L = nullptr;
  const int nslots = 3;
  if (rkl_create(&L, 2, bases, rb, nrows, 4, nslots) || !L) return 2;
  std::mt19937 rng(1);
  const int64_t batch = 257;
  std::vector<std::vector<int64_t>> idx(nslots, std::vector<int64_t>(batch));
  std::vector<std::vector<std::vector<unsigned char>>> out(nslots, std::vector<std::vector<unsigned char>>(2));
  for (int s = 0; s < nslots; ++s)
    for (int t = 0; t < 2; ++t) out[s][t].resize(batch * rb[t]);
  int bad = 0;
  for (int it = 0; it < 60; ++it) {
    const int s = it % nslots;
    if (it >= nslots) {  // verify this slot's previous job before reusing it
      rkl_wait(L, s);
      for (int64_t r = 0; r < batch; ++r)
        for (int t = 0; t < 2; ++t)
          bad += std::memcmp(out[s][t].data() + r * rb[t], data[t].data() + idx[s][r] * rb[t], rb[t]) != 0;
    }
    for (auto& v : idx[s]) v = (int64_t)(rng() % nrows);
    void* dst[2] = {out[s][0].data(), out[s][1].data()};
    if (rkl_submit(L, s, idx[s].data(), batch, dst)) return 3;
  }
  rkl_destroy(L);  // waits for the jobs still in flight
  std::printf("loader stress: %d bad rows\n", bad);
  return bad ? 1 : 0;
}

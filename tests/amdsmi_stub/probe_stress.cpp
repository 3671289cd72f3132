// Concurrency driver for csrc/probe/probe.cpp under ThreadSanitizer (tests/test_sanitizers.py).
//
// The agent calls the probe's C ABI from its main loop while /probe and /metrics handlers and the
// checker's fan-out can hit it from other threads; the Python binding releases the GIL around every
// ctypes call.  Here T threads interleave open / json / gpu_count / close for R rounds each against the
// replay stub of libamd_smi; every document must parse as one "mi355x-health/v1" object.
//
//   probe_stress THREADS ROUNDS
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "probe.h"

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 8;
  const int rounds = argc > 2 ? atoi(argv[2]) : 50;
  std::vector<std::thread> ts;
  std::vector<int> bad(static_cast<size_t>(threads), 0);
  for (int t = 0; t < threads; ++t) {
    ts.emplace_back([t, rounds, &bad] {
      for (int r = 0; r < rounds; ++r) {
        if ((r + t) % 7 == 0) mi355x_probe_open();
        char* doc = mi355x_probe_json("stress-node");
        if (!doc || strncmp(doc, "{\"schema\":\"mi355x-health/v1\"", 28) != 0 || doc[strlen(doc) - 1] != '}')
          ++bad[static_cast<size_t>(t)];
        mi355x_probe_free(doc);
        (void)mi355x_probe_gpu_count();
        if (t == 0 && r % 10 == 9) mi355x_probe_close();  // re-initialised by the next call
      }
    });
  }
  for (auto& th : ts) th.join();
  mi355x_probe_close();
  int nbad = 0;
  for (int b : bad) nbad += b;
  printf("{\"threads\":%d,\"rounds\":%d,\"bad_documents\":%d,\"gpus\":%d}\n", threads, rounds, nbad,
         mi355x_probe_gpu_count());
  return nbad ? 1 : 0;
}

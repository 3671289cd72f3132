// mi355x-probe: standalone CLI around probe.cpp for DaemonSets without Python.
//
//   mi355x-probe [--node NAME] [--repeat N] [--interval-ms MS]
//
// Prints one "mi355x-health/v1" JSON document per probe on stdout.  Exit code:
// 0 probe ran, 1 amd-smi could not be initialised (the JSON still says why).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>

#include "probe.h"

int main(int argc, char** argv) {
  std::string node;
  int repeat = 1;
  int interval_ms = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--node") && i + 1 < argc) {
      node = argv[++i];
    } else if (!strcmp(argv[i], "--repeat") && i + 1 < argc) {
      repeat = atoi(argv[++i]);
    } else if (!strcmp(argv[i], "--interval-ms") && i + 1 < argc) {
      interval_ms = atoi(argv[++i]);
    } else {
      fprintf(stderr, "usage: %s [--node NAME] [--repeat N] [--interval-ms MS]\n", argv[0]);
      return 2;
    }
  }
  if (node.empty()) {
    const char* env = getenv("NODE_NAME");
    if (env) {
      node = env;
    } else {
      char host[256] = {0};
      gethostname(host, sizeof host - 1);
      node = host;
    }
  }
  int rc = mi355x_probe_open();
  for (int r = 0; r < repeat; ++r) {
    char* doc = mi355x_probe_json(node.c_str());
    if (doc) {
      puts(doc);
      fflush(stdout);
      mi355x_probe_free(doc);
    }
    if (interval_ms > 0 && r + 1 < repeat) std::this_thread::sleep_for(std::chrono::milliseconds(interval_ms));
  }
  mi355x_probe_close();
  return rc == 0 ? 0 : 1;
}

// Fault injection for the native collectives — the C++ twin of
// utils/faults.py, reading the same CS744_FAULT spec so one environment variable drives
// both the torch.distributed facade and the engine's stream-ordered communicators:
//   CS744_FAULT="<op>[@N]:<rank>:<action>[:<arg>]"[,...]
// op: all_reduce | broadcast | * ; rank: an int or * ; @N fires only at the N-th matching
// call; action: kill (exit 17 without unwinding, like a crashed rank), delay (sleep arg
// seconds on the host before enqueueing), raise (std::runtime_error -> Python RuntimeError).
// The reference has no fault handling at all (it relies on gloo's 30-minute default,
// master/part2a/part2a.py:84).
#pragma once
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace cs {

inline void fault_point(const char* op, int rank) {
  static std::map<std::string, int> counts;
  const char* env = getenv("CS744_FAULT");
  if (env == nullptr || *env == 0) return;
  std::stringstream all(env);
  std::string one;
  while (std::getline(all, one, ',')) {
    std::vector<std::string> f;
    std::stringstream ss(one);
    std::string tok;
    while (std::getline(ss, tok, ':')) f.push_back(tok);
    if (f.size() < 3) throw std::runtime_error("bad CS744_FAULT spec " + one);
    std::string fop = f[0];
    int nth = -1;
    const size_t at = fop.find('@');
    if (at != std::string::npos) {
      nth = atoi(fop.c_str() + at + 1);
      fop = fop.substr(0, at);
    }
    if (fop != "*" && fop != op) continue;
    if (f[1] != "*" && atoi(f[1].c_str()) != rank) continue;
    const int n = ++counts[fop + ":" + f[1]];
    if (nth >= 0 && n != nth) continue;
    if (f[2] == "kill") {
      fprintf(stderr, "[fault] rank %d: killing at native %s\n", rank, op);
      fflush(stderr);
      _Exit(17);
    } else if (f[2] == "delay") {
      const double s = f.size() > 3 ? atof(f[3].c_str()) : 1.0;
      std::this_thread::sleep_for(std::chrono::duration<double>(s));
    } else if (f[2] == "raise") {
      throw std::runtime_error(std::string("[fault] injected failure at native ") + op + " on rank " +
                               std::to_string(rank));
    } else {
      throw std::runtime_error("unknown fault action " + f[2]);
    }
  }
}

}  // namespace cs

// jit.cpp — compiles a query's generated NFA step policy (compile.cpp generate_jit) with
// hipRTC for gfx950 and loads it as a module.  Code objects are cached on disk by a hash of
// the source and options ($CEP_JIT_CACHE, default <libcep dir>/jit_cache), so a query is
// compiled once per machine; build() pre-populates the cache for the benchmark queries.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <utime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "cep_internal.h"
#include "jit_headers.inc"

namespace cep {

namespace {

// stand-ins for the two system headers the shared device headers include: hipRTC supplies
// the HIP device runtime itself and the fixed-width types under __hip_internal
const char* kStdint = R"(#pragma once
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::int16_t int16_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::int8_t int8_t;
#define INT64_MAX 0x7fffffffffffffffLL
#define INT64_MIN (-INT64_MAX - 1)
#define INT32_MAX 0x7fffffff
#define INT32_MIN (-INT32_MAX - 1)
)";
const char* kHipRuntime = "#pragma once\n";

const char* kOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off"};

// compile options: kOpts, then (measurement builds) $CEP_JIT_OPTS split on spaces (compiler
// scheduling strategies and the like; part of the cache key)
std::vector<std::string> jit_opts() {
  std::vector<std::string> o(std::begin(kOpts), std::end(kOpts));
#ifdef CEP_MEASURE
  if (const char* e = std::getenv("CEP_JIT_OPTS")) {
    std::string cur;
    for (const char* c = e;; c++) {
      if (*c == ' ' || *c == 0) {
        if (!cur.empty()) o.push_back(cur);
        cur.clear();
        if (*c == 0) break;
      } else {
        cur += *c;
      }
    }
  }
#endif
  return o;
}

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

std::string cache_dir() {
  if (const char* e = std::getenv("CEP_JIT_CACHE")) return e;
  Dl_info info{};
  if (dladdr((void*)&fnv1a, &info) && info.dli_fname) {
    std::string p = info.dli_fname;
    auto k = p.rfind('/');
    if (k != std::string::npos) return p.substr(0, k) + "/jit_cache";
  }
  return "/tmp/cep_jit_cache";
}

std::mutex g_mu;

}  // namespace

std::string jit_cache_key(const std::string& src) {
  std::string all = src;
  for (const auto& o : jit_opts()) all += o;
  for (int i = 0; i < kJitHeaderCount; i++) all += kJitHeaderSrcs[i];
  char b[32];
  std::snprintf(b, sizeof b, "%016llx", (unsigned long long)fnv1a(all));
  return b;
}

// Returns the gfx950 code object for `src`, from the cache or freshly compiled.  `touch`: a
// cache hit refreshes its entry's mtime (cep_jit_precompile*: tests/precompile_jit.py drops the
// entries no current query maps to by their mtime).
std::vector<char> jit_code_object(const std::string& src, double* compile_s, bool touch) {
  std::lock_guard<std::mutex> lk(g_mu);
  const std::string dir = cache_dir();
  const std::string path = dir + "/" + jit_cache_key(src) + ".co";
  if (compile_s) *compile_s = 0;
  {
    std::ifstream f(path, std::ios::binary);
    if (f) {
      std::vector<char> co((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
      if (!co.empty()) {
        if (touch) utime(path.c_str(), nullptr);
        return co;
      }
    }
  }
  std::vector<const char*> names, srcs;
  names.push_back("stdint.h");
  srcs.push_back(kStdint);
  names.push_back("hip/hip_runtime.h");
  srcs.push_back(kHipRuntime);
  for (int i = 0; i < kJitHeaderCount; i++) {
    names.push_back(kJitHeaderNames[i]);
    srcs.push_back(kJitHeaderSrcs[i]);
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "cep_query.hip", (int)names.size(), srcs.data(), names.data()) !=
      HIPRTC_SUCCESS)
    throw std::runtime_error("hiprtcCreateProgram failed");
  auto t0 = std::chrono::steady_clock::now();
  const std::vector<std::string> opts = jit_opts();
  std::vector<const char*> optv;
  for (const auto& o : opts) optv.push_back(o.c_str());
  const hiprtcResult rc = hiprtcCompileProgram(prog, (int)optv.size(), optv.data());
  if (compile_s) *compile_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    throw std::runtime_error("query JIT compile failed: " + log.substr(0, 4000));
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  std::vector<char> co(n);
  hiprtcGetCode(prog, co.data());
  hiprtcDestroyProgram(&prog);
  mkdir(dir.c_str(), 0755);
  const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
  {
    std::ofstream f(tmp, std::ios::binary);
    f.write(co.data(), (std::streamsize)co.size());
  }
  std::rename(tmp.c_str(), path.c_str());
  return co;
}

}  // namespace cep

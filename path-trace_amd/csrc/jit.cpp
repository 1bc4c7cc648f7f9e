/*
 * jit.cpp -- compiles generated scene modules for gfx950 with hiprtc and keeps
 * the code objects in an on-disk cache (default: path-trace_amd/_jit_cache
 * next to libpt.so, overridable with PT_JIT_CACHE).  build() pre-populates the
 * cache for the benchmark scenes so the GPU box only loads code objects; an
 * unseen scene is compiled on first use (no GPU needed to compile).
 */
#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <utime.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <mutex>
#include <sstream>

#include "internal.h"

namespace pt
{

namespace
{

const char *kOptions[] = {
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",                           /* no FMA contraction: bit parity with the x86 reference */
    "-fhip-fp32-correctly-rounded-divide-sqrt",    /* IEEE-exact f32 '/' and sqrt                           */
    "-fno-gpu-flush-denormals-to-zero",           /* keep f32 denormals as the reference does              */
    "-fno-fast-math",
};

std::string cache_dir()
{
    const char *env = getenv("PT_JIT_CACHE");
    if (env && *env)
        return env;
    Dl_info info;
    if (dladdr((void *)&cache_dir, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        size_t k = p.find_last_of('/');
        std::string dir = k == std::string::npos ? "." : p.substr(0, k);
        return dir + "/../_jit_cache";
    }
    return "./_jit_cache";
}

std::string full_key(const Generated &g)
{
    int maj = 0, min = 0;
    hiprtcVersion(&maj, &min);
    std::ostringstream k;
    k << g.source << "\n";
    for (const char *o : kOptions) k << o << "\n";
    k << "hiprtc " << maj << "." << min << "\n";
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : k.str()) {
        h ^= c;
        h *= 1099511628211ull;
    }
    char buf[40];
    snprintf(buf, sizeof buf, "%016llx", (unsigned long long)h);
    return buf;
}

std::mutex g_mu;
std::map<std::string, std::vector<char>> g_mem;

std::vector<char> compile(const Generated &g, std::string &log)
{
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, g.source.c_str(), "pt_scene.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        throw Error(PT_ERR_COMPILE, "hiprtcCreateProgram failed");
    int n = (int)(sizeof(kOptions) / sizeof(kOptions[0]));
    hiprtcResult r = hiprtcCompileProgram(prog, n, kOptions);
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    log.assign(ls, '\0');
    if (ls)
        hiprtcGetProgramLog(prog, &log[0]);
    if (r != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        throw Error(PT_ERR_COMPILE, "hiprtc compile failed: " + log.substr(0, 4000));
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    std::vector<char> code(cs);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    return code;
}

} // namespace

const std::vector<char> &code_object(const Generated &g)
{
    std::lock_guard<std::mutex> lk(g_mu);
    std::string key = full_key(g);
    auto it = g_mem.find(key);
    if (it != g_mem.end())
        return it->second;
    std::string dir = cache_dir();
    std::string path = dir + "/" + key + ".hsaco";
    {
        std::ifstream f(path, std::ios::binary);
        if (f) {
            std::vector<char> code((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
            if (!code.empty()) {
                utime(path.c_str(), nullptr); /* mark as used (build() prunes unused objects) */
                return g_mem[key] = std::move(code);
            }
        }
    }
    std::string log;
    std::vector<char> code = compile(g, log);
    mkdir(dir.c_str(), 0755);
    std::string tmp = path + ".tmp" + std::to_string(getpid());
    {
        std::ofstream f(tmp, std::ios::binary);
        f.write(code.data(), (std::streamsize)code.size());
    }
    if (rename(tmp.c_str(), path.c_str()) != 0)
        unlink(tmp.c_str());
    /* keep the generated source beside the code object for inspection */
    std::ofstream(dir + "/" + key + ".hip") << g.source;
    return g_mem[key] = std::move(code);
}

} // namespace pt

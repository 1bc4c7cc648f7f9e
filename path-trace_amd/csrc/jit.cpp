/*
 * jit.cpp -- compiles generated scene modules for gfx950 with hiprtc and keeps
 * the code objects in an on-disk cache (default: path-trace_amd/_jit_cache
 * next to libpt.so, overridable with PT_JIT_CACHE).  build() pre-populates the
 * cache for the benchmark scenes so the GPU box only loads code objects; an
 * unseen scene is compiled on first use (no GPU needed to compile).
 *
 * hiprtc is dlopen'ed by absolute path ($ROCM_PATH or /opt/rocm) rather than
 * linked: a PyTorch process already holds torch's own libhiprtc.so (soname
 * libhiprtc.so.7, an older compiler), which a plain NEEDED entry would bind
 * to whenever torch is imported first -- the code objects would then depend
 * on import order.  The HIP runtime itself (libamdhip64.so.7) is deliberately
 * the process's one, so device pointers and streams from torch are valid here.
 */
#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <utime.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <mutex>
#include <sstream>

#include "internal.h"

namespace pt
{

namespace
{

struct Rtc
{
    decltype(&hiprtcCreateProgram) create;
    decltype(&hiprtcCompileProgram) compile;
    decltype(&hiprtcGetProgramLogSize) log_size;
    decltype(&hiprtcGetProgramLog) log;
    decltype(&hiprtcGetCodeSize) code_size;
    decltype(&hiprtcGetCode) code;
    decltype(&hiprtcDestroyProgram) destroy;
    decltype(&hiprtcVersion) version;
};

const Rtc &rtc()
{
    static Rtc r = [] {
        std::string root = getenv("ROCM_PATH") && *getenv("ROCM_PATH") ? getenv("ROCM_PATH") : "/opt/rocm";
        std::string path = root + "/lib/libhiprtc.so.7";
        void *h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h)
            throw Error(PT_ERR_COMPILE, "cannot load " + path + ": " + dlerror());
        Rtc t;
        auto sym = [&](const char *n) {
            void *p = dlsym(h, n);
            if (!p)
                throw Error(PT_ERR_COMPILE, std::string("hiprtc symbol missing: ") + n);
            return p;
        };
        t.create = (decltype(t.create))sym("hiprtcCreateProgram");
        t.compile = (decltype(t.compile))sym("hiprtcCompileProgram");
        t.log_size = (decltype(t.log_size))sym("hiprtcGetProgramLogSize");
        t.log = (decltype(t.log))sym("hiprtcGetProgramLog");
        t.code_size = (decltype(t.code_size))sym("hiprtcGetCodeSize");
        t.code = (decltype(t.code))sym("hiprtcGetCode");
        t.destroy = (decltype(t.destroy))sym("hiprtcDestroyProgram");
        t.version = (decltype(t.version))sym("hiprtcVersion");
        return t;
    }();
    return r;
}

const char *kOptions[] = {
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",                           /* no FMA contraction: bit parity with the x86 reference */
    "-fhip-fp32-correctly-rounded-divide-sqrt",    /* IEEE-exact f32 '/' and sqrt                           */
    "-fno-gpu-flush-denormals-to-zero",           /* keep f32 denormals as the reference does              */
    "-fno-fast-math",
    "-fno-slp-vectorize", /* packing pairs of f32 ops into v_pk_* costs more v_mov than it saves (A/B on C3) */
    /* live-range splitting around spills sized for fewer copies: the megakernel
     * spills at every occupancy (A/B on one box: C3 120.5 -> 124.5 Msamples/s,
     * C2 and C5 unchanged within noise) */
    "-mllvm",
    "-split-spill-mode=size",
    /* no unclustered high-register-pressure rescheduling stage: same-box A/B,
     * profiles/round4/ab_sched_options_*.txt: C2 +1.4 %, C5 +0.1 %, C3 +-0
     * (max-ilp scheduling: C3 -5.5 %; the AMDGPU RP trackers: +-0.5 %) */
    "-mllvm",
    "-amdgpu-disable-unclustered-high-rp-reschedule",
    /* LDS is sized by hand for the workgroups-per-CU target (min_workgroups);
     * private arrays the promoter would move into spare LDS can push a
     * workgroup past the CU's 160 KB / 1280-B granule budget */
    "-mllvm",
    "-disable-promote-alloca-to-lds",
};

/* experiment hook: extra compiler options, e.g. PT_JIT_OPTIONS="-fno-slp-vectorize".
 * Options that change floating-point semantics would silently break the
 * bit-exact contract and are refused; an active hook is announced on stderr. */
std::vector<std::string> extra_options()
{
    static const std::vector<std::string> v = [] {
        std::vector<std::string> r;
        const char *env = getenv("PT_JIT_OPTIONS");
        if (!env || !*env)
            return r;
        static const char *banned[] = {"fast-math", "Ofast", "fp-contract", "denormal", "flush", "finite-math",
                                       "unsafe", "associative", "reciprocal", "signed-zeros", "approx",
                                       "correctly-rounded", "fp-model", "ffp-"};
        std::istringstream in(env);
        std::string o;
        while (in >> o) {
            for (const char *b : banned)
                if (o.find(b) != std::string::npos)
                    throw Error(PT_ERR_ARG, "PT_JIT_OPTIONS: '" + o + "' would change floating-point semantics");
            r.push_back(o);
        }
        fprintf(stderr, "pt: experiment hook PT_JIT_OPTIONS=\"%s\" active\n", env);
        return r;
    }();
    return v;
}

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
    rtc().version(&maj, &min);
    std::ostringstream k;
    k << g.source << "\n";
    for (const char *o : kOptions) k << o << "\n";
    for (const std::string &o : g.options) k << o << "\n";
    for (const std::string &o : extra_options()) k << o << "\n";
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
    const Rtc &R = rtc();
    hiprtcProgram prog;
    if (R.create(&prog, g.source.c_str(), "pt_scene.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        throw Error(PT_ERR_COMPILE, "hiprtcCreateProgram failed");
    std::vector<const char *> opts(std::begin(kOptions), std::end(kOptions));
    for (const std::string &o : g.options)
        opts.push_back(o.c_str());
    const std::vector<std::string> extra = extra_options();
    for (const std::string &o : extra)
        opts.push_back(o.c_str());
    hiprtcResult r = R.compile(prog, (int)opts.size(), opts.data());
    size_t ls = 0;
    R.log_size(prog, &ls);
    log.assign(ls, '\0');
    if (ls)
        R.log(prog, &log[0]);
    if (r != HIPRTC_SUCCESS) {
        R.destroy(&prog);
        throw Error(PT_ERR_COMPILE, "hiprtc compile failed: " + log.substr(0, 4000));
    }
    size_t cs = 0;
    R.code_size(prog, &cs);
    std::vector<char> code(cs);
    R.code(prog, code.data());
    R.destroy(&prog);
    return code;
}

} // namespace

std::string code_object_key(const Generated &g) { return full_key(g); }

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

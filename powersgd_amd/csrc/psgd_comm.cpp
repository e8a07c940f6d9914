// RCCL inside libpsgd: communicators and the stream-ordered SUM all-reduce of a world-size-W
// step (psgd_aggregate_comm, psgd_plan.cpp). RCCL is resolved at run time with dlopen/dlsym
// (psgd_comm_* in include/psgd.h): an RCCL the process has already loaded (PyTorch's) is reused,
// else PSGD_RCCL_LIB or the ROCm one; the library has no link-time dependency on it.
// PSGD_RCCL_LIB_FORCE=<path> (tests only) takes precedence over all of these and is read at
// every psgd_comm_unique_id / psgd_comm_init: each communicator keeps the function table of the
// library it was created with, so one process can hold a real and a stand-in communicator
// (tests/stubs/rccl_stub.hip drives psgd_aggregate_comm at world size W on one GPU). The override
// needs a second, explicit opt-in (PSGD_TESTING=1) and announces itself on stderr once per
// library: a stray PSGD_RCCL_LIB_FORCE in a training job's environment is ignored (with a
// warning) instead of silently replacing RCCL.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "psgd.h"
#include "psgd_internal.h"

namespace psgd {
namespace {
struct Rccl;
}
}  // namespace psgd

struct psgd_comm {
    const psgd::Rccl* lib = nullptr;  // the collective library this communicator was created with
    ncclComm_t comm = nullptr;
    int world = 0, rank = -1, device = -1;
    // set by the first failed collective: the ranks' call sequences have diverged, so every
    // later call fails at once (PSGD_ERR_STATE) instead of enqueueing into a communicator whose
    // peers are waiting on a different collective (a hang elsewhere)
    bool poisoned = false;
    std::string poison;
};

namespace psgd {
namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string error;
};

Rccl load(const char* forced) {
    Rccl r;
    void* h = nullptr;
    if (forced) {
        h = dlopen(forced, RTLD_NOW | RTLD_LOCAL);
    } else {
        // 1. an RCCL already in the process (the host framework's), 2. PSGD_RCCL_LIB, 3. ROCm's
        for (const char* name : {"librccl.so", "librccl.so.1"}) {
            if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
        }
        const char* env = std::getenv("PSGD_RCCL_LIB");
        if (!h && env && *env) h = dlopen(env, RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    }
    if (!h) {
        const char* de = dlerror();  // read once: a second call returns null
        r.error = std::string("cannot load ") + (forced ? forced : "librccl.so") + ": " + (de ? de : "?");
        return r;
    }
    auto sym = [&](const char* n) { return dlsym(h, n); };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<decltype(r.init_rank)>(sym("ncclCommInitRank"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(sym("ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    if (!r.get_unique_id || !r.init_rank || !r.destroy || !r.all_reduce || !r.group_start || !r.group_end ||
        !r.error_string)
        r.error = "librccl.so lacks an expected symbol";
    return r;
}

// The library for a new communicator: PSGD_RCCL_LIB_FORCE if set together with PSGD_TESTING=1
// (tests), else the process's RCCL. Tables live for the whole process (communicators point at
// them).
const Rccl& rccl() {
    static std::mutex mu;
    static std::map<std::string, std::unique_ptr<Rccl>> libs;
    const char* forced = std::getenv("PSGD_RCCL_LIB_FORCE");
    if (forced && !*forced) forced = nullptr;
    const char* testing = std::getenv("PSGD_TESTING");
    const bool opted_in = testing && std::strcmp(testing, "1") == 0;
    std::lock_guard<std::mutex> lock(mu);
    if (forced && !opted_in) {
        static bool warned = false;
        if (!warned)
            std::fprintf(stderr, "libpsgd: PSGD_RCCL_LIB_FORCE=%s ignored (test-only override; needs PSGD_TESTING=1)\n",
                         forced);
        warned = true;
        forced = nullptr;
    }
    std::unique_ptr<Rccl>& slot = libs[forced ? std::string(forced) : std::string()];
    if (!slot) {
        if (forced)
            std::fprintf(stderr, "libpsgd: collective library replaced by %s (PSGD_RCCL_LIB_FORCE, tests only)\n",
                         forced);
        slot.reset(new Rccl(load(forced)));
    }
    return *slot;
}

int rccl_fail(const Rccl& r, ncclResult_t e, const char* what) {
    return comm_fail(PSGD_ERR_DEVICE, (std::string(what) + ": " + (r.error_string ? r.error_string(e) : "?")).c_str());
}

}  // namespace

int comm_world(const psgd_comm* c) { return c->world; }

bool comm_poisoned(const psgd_comm* c, std::string* why) {
    if (c->poisoned && why) *why = c->poison;
    return c->poisoned;
}

void comm_poison(psgd_comm* c, const char* why) {
    if (c->poisoned) return;
    c->poisoned = true;
    c->poison = why ? why : "?";
}

int comm_allreduce(psgd_comm* c, float* buf, size_t n, float* buf2, size_t n2, hipStream_t s) {
    const Rccl& r = *c->lib;
    if (!r.error.empty()) return comm_fail(PSGD_ERR_STATE, r.error.c_str());
    if (c->poisoned) return comm_fail(PSGD_ERR_STATE, ("communicator unusable after an earlier failure: " + c->poison).c_str());
    ncclResult_t e = ncclSuccess;
    const char* what = "ncclAllReduce";
    if (!(n && n2)) {  // one collective: no group calls around it
        if (n) e = r.all_reduce(buf, buf, n, ncclFloat32, ncclSum, c->comm, s);
        else if (n2) e = r.all_reduce(buf2, buf2, n2, ncclFloat32, ncclSum, c->comm, s);
    } else {
        e = r.group_start();
        what = "ncclGroupStart";
        if (e == ncclSuccess) {
            what = "ncclAllReduce";
            e = r.all_reduce(buf, buf, n, ncclFloat32, ncclSum, c->comm, s);
            if (e == ncclSuccess) e = r.all_reduce(buf2, buf2, n2, ncclFloat32, ncclSum, c->comm, s);
            const ncclResult_t e2 = r.group_end();
            if (e == ncclSuccess && e2 != ncclSuccess) {
                e = e2;
                what = "ncclGroupEnd";
            }
        }
    }
    if (e != ncclSuccess) {
        c->poisoned = true;
        c->poison = std::string(what) + ": " + (r.error_string ? r.error_string(e) : "?");
        return rccl_fail(r, e, what);
    }
    return PSGD_OK;
}

}  // namespace psgd

using namespace psgd;

extern "C" {

int psgd_comm_id_bytes(int64_t* bytes) {
    if (!bytes) return comm_fail(PSGD_ERR_VALUE, "null argument");
    *bytes = int64_t(sizeof(ncclUniqueId));
    return PSGD_OK;
}

int psgd_comm_unique_id(void* id_out) {
    if (!id_out) return comm_fail(PSGD_ERR_VALUE, "null argument");
    const Rccl& r = rccl();
    if (!r.error.empty()) return comm_fail(PSGD_ERR_STATE, r.error.c_str());
    ncclUniqueId id;
    const ncclResult_t e = r.get_unique_id(&id);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof(id));
    return PSGD_OK;
}

int psgd_comm_init(int32_t world, int32_t rank, const void* id, int32_t device, psgd_comm** out) {
    if (!id || !out) return comm_fail(PSGD_ERR_VALUE, "null argument");
    *out = nullptr;
    if (world < 1 || rank < 0 || rank >= world) return comm_fail(PSGD_ERR_VALUE, "bad world/rank");
    const Rccl& r = rccl();
    if (!r.error.empty()) return comm_fail(PSGD_ERR_STATE, r.error.c_str());
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (device >= 0) (void)hipSetDevice(device);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    auto* c = new psgd_comm();
    const ncclResult_t e = r.init_rank(&c->comm, world, uid, rank);
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    if (e != ncclSuccess) {
        delete c;
        return rccl_fail(r, e, "ncclCommInitRank");
    }
    c->lib = &r;
    c->world = world;
    c->rank = rank;
    c->device = device;
    *out = c;
    return PSGD_OK;
}

int psgd_comm_destroy(psgd_comm* c) {
    if (!c) return PSGD_OK;
    if (c->comm && c->lib) (void)c->lib->destroy(c->comm);
    delete c;
    return PSGD_OK;
}

}  // extern "C"

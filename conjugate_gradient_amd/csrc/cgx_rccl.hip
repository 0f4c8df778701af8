// cgx_rccl.hip -- RCCL loaded on first use (cgx_ctx.h).  Only rank mode
// (cgx_create_rank*, cgx_get_unique_id) talks to RCCL; loading it with the
// library made every process's HIP start-up ~25-35 ms longer (its device
// code registers with the runtime; profiles/r01_hip_init_rccl.txt), so
// single-GPU and multi-shard use, the CLI included, never load it.  If the
// process already has librccl.so.1 (torch's), dlopen returns that one.  The
// load is attempted once per process: a failure is permanent (every later
// rank-mode call returns CGX_ERR_RCCL with the same reason).
#include <dlfcn.h>

#include <cstdlib>
#include <mutex>
#include <type_traits>

#define CGX_RCCL_LOADER
#include "cgx_ctx.h"

namespace cgxh {

RcclApi g_rccl;

bool rccl_load() {
    static std::once_flag once;
    static bool ok = false;
    static char why[512] = "";
    std::call_once(once, [] {
        // soname first (the one torch already mapped, if any), then
        // $ROCM_PATH/lib, then the image's /opt/rocm.  RTLD_LOCAL: every symbol
        // is taken through this handle, and a later torch import must not bind
        // to it by accident.
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            if (const char *rp = std::getenv("ROCM_PATH")) {
                char path[1024];
                snprintf(path, sizeof path, "%s/lib/librccl.so.1", rp);
                h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
            }
        }
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char *e = dlerror();
            snprintf(why, sizeof why, "%s", e ? e : "dlopen failed");
            return;
        }
        bool all = true;
        auto get = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) {
                all = false;
                snprintf(why, sizeof why, "librccl.so.1 has no %s", name);
            }
        };
        get(g_rccl.GetUniqueId, "ncclGetUniqueId");
        get(g_rccl.CommInitRank, "ncclCommInitRank");
        get(g_rccl.CommDestroy, "ncclCommDestroy");
        get(g_rccl.GetErrorString, "ncclGetErrorString");
        get(g_rccl.AllGather, "ncclAllGather");
        get(g_rccl.AllReduce, "ncclAllReduce");
        get(g_rccl.Send, "ncclSend");
        get(g_rccl.Recv, "ncclRecv");
        get(g_rccl.GroupStart, "ncclGroupStart");
        get(g_rccl.GroupEnd, "ncclGroupEnd");
        get(g_rccl.CommGetAsyncError, "ncclCommGetAsyncError");
        get(g_rccl.CommAbort, "ncclCommAbort");
        get(g_rccl.CommCount, "ncclCommCount");
        get(g_rccl.CommCuDevice, "ncclCommCuDevice");
        get(g_rccl.CommUserRank, "ncclCommUserRank");
        ok = all;
    });
    if (!ok) fail(CGX_ERR_RCCL, "cannot load RCCL: %s", why);
    return ok;
}

}  // namespace cgxh

// dist.cpp — the multi-GPU data path behind the C ABI (include/sdrg.h, "Multi-GPU"): one process per GPU, the
// streams sharded contiguously over the ranks (rank r owns global streams [r*B, (r+1)*B)), and the one collective of
// the path -- the per-frame results of every rank gathered to a root rank -- as RCCL ncclGather over xGMI, enqueued
// on the engine stream that produced the gathered outputs (engine.cpp, sdrg_engine_gather), so that it follows each
// call's kernels without a host synchronisation.
//
// What the gather carries is what the reference's soapyCallback hands to Kotlin per frame
// (src/sdr-bridge-java-soapy.cpp:456-466: the fftCallback spectrum, then the getters' values -- here the 72-byte
// sdrg_frame_record with the peak index) and the SSB worker's PCM (src/ssb/ssb_processor.cpp:103-108); SURVEY.md 8e
// sizes them.  The reference itself is single-process (one receiver); the sharding is this build's.
//
// RCCL is loaded at run time (dlopen of librccl.so.1, the soname both /opt/rocm/lib and PyTorch ship, so a process
// that already holds PyTorch's RCCL uses that one instance), the first time a communicator is made: the library
// loads and runs everything else without RCCL present.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <mutex>
#include <string>

#include "sdrg_internal.h"

using namespace sdrg;

namespace {

struct RcclApi {
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*get_version)(int *) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    std::string error;  // empty when every symbol resolved
};

const RcclApi &rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char *m = dlerror();
            api.error = std::string("cannot load librccl.so.1: ") + (m ? m : "?");
            return;
        }
        auto sym = [&](const char *name, auto &fp) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            if (!fp && api.error.empty()) api.error = std::string("librccl.so.1 lacks ") + name;
        };
        sym("ncclGetUniqueId", api.get_unique_id);
        sym("ncclCommInitRank", api.comm_init_rank);
        sym("ncclCommDestroy", api.comm_destroy);
        sym("ncclGather", api.gather);
        sym("ncclGroupStart", api.group_start);
        sym("ncclGroupEnd", api.group_end);
        sym("ncclGetVersion", api.get_version);
        sym("ncclGetErrorString", api.error_string);
    });
    return api;
}

// SDRG_OK if `device` names a HIP device of this process, else the failure (message via sdrg_last_error)
int32_t check_device(int32_t device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(SDRG_E_NODEVICE, "no HIP device");
    if (device < 0 || device >= count) return fail(SDRG_E_INVALID, "device %d out of range [0, %d)", device, count);
    return SDRG_OK;
}

int32_t rccl_fail(const RcclApi &a, ncclResult_t r, const char *what) {
    return fail(SDRG_E_HIP, "%s: %s", what, a.error_string ? a.error_string(r) : "RCCL error");
}

}  // namespace

struct sdrg_dist {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 0, device = 0;
    bool rccl_data = true;  // the gathers go through RCCL (false: a one-rank communicator's device copies)
};

// A one-rank gather is a copy.  RCCL runs it as its generic kernel (5 workgroups, 141 us on average beside the SSB
// pipeline in bench.py --process-group, rocprofv3 r5p), whose waves slow the CUs they land on, and a persistent pipeline
// runs at its slowest CU's pace: the c3 step +2.8 % for the 288-KB records gather.  So at world size 1 the gathers are
// hipMemcpyAsync device copies on the same stream (a ~3 us blit); sdrg_dist_set_one_rank_rccl(d, 1) keeps RCCL there
// too (tests/test_gpu_dist_capi.py runs both).

int32_t sdrg::dist_gather(sdrg_dist *d, const GatherItem *items, int n_items, int root, hipStream_t stream) {
    const RcclApi &a = rccl();
    if (!a.error.empty()) return fail(SDRG_E_UNSUPPORTED, "%s", a.error.c_str());
    if (root < 0 || root >= d->world) return fail(SDRG_E_INVALID, "root %d outside [0, %d)", root, d->world);
    for (int i = 0; i < n_items; i++)
        if (!items[i].send || (d->rank == root && !items[i].recv))
            return fail(SDRG_E_INVALID, "gather item %d: null %s buffer", i, items[i].send ? "receive" : "send");
    if (!d->rccl_data) {  // world size 1: the root's own blocks
        for (int i = 0; i < n_items; i++)
            if (items[i].bytes && items[i].recv != items[i].send) {
                hipError_t e = hipMemcpyAsync(items[i].recv, items[i].send, items[i].bytes, hipMemcpyDeviceToDevice, stream);
                if (e != hipSuccess) return fail(SDRG_E_HIP, "hipMemcpyAsync: %s", hipGetErrorString(e));
            }
        return SDRG_OK;
    }
    // one group: every selected gather goes out as one RCCL launch on the stream
    ncclResult_t r = a.group_start();
    if (r != ncclSuccess) return rccl_fail(a, r, "ncclGroupStart");
    ncclResult_t first = ncclSuccess;
    for (int i = 0; i < n_items; i++) {
        r = a.gather(items[i].send, d->rank == root ? items[i].recv : nullptr, items[i].bytes, ncclUint8, root, d->comm,
                     stream);
        if (r != ncclSuccess && first == ncclSuccess) first = r;
    }
    r = a.group_end();
    if (first != ncclSuccess) return rccl_fail(a, first, "ncclGather");
    if (r != ncclSuccess) return rccl_fail(a, r, "ncclGroupEnd");
    return SDRG_OK;
}

int sdrg::dist_device(const sdrg_dist *d) { return d->device; }
int sdrg::dist_world(const sdrg_dist *d) { return d->world; }
int sdrg::dist_rank(const sdrg_dist *d) { return d->rank; }

extern "C" {

int32_t sdrg_dist_unique_id(void *id, int32_t bytes) {
    if (!id || bytes < SDRG_DIST_ID_BYTES) return fail(SDRG_E_INVALID, "id buffer must hold %d bytes", SDRG_DIST_ID_BYTES);
    const RcclApi &a = rccl();
    if (!a.error.empty()) return fail(SDRG_E_UNSUPPORTED, "%s", a.error.c_str());
    static_assert(sizeof(ncclUniqueId) == SDRG_DIST_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    ncclResult_t r = a.get_unique_id(&u);
    if (r != ncclSuccess) return rccl_fail(a, r, "ncclGetUniqueId");
    memcpy(id, &u, sizeof(u));
    return SDRG_OK;
}

int32_t sdrg_dist_create(const void *id, int32_t world_size, int32_t rank, int32_t device, sdrg_dist **out) {
    if (!out) return fail(SDRG_E_INVALID, "null out");
    *out = nullptr;
    if (!id) return fail(SDRG_E_INVALID, "null id");
    if (world_size < 1 || rank < 0 || rank >= world_size)
        return fail(SDRG_E_INVALID, "rank %d / world_size %d", rank, world_size);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(SDRG_E_NODEVICE, "no HIP device");
    if (device < 0 || device >= count) return fail(SDRG_E_INVALID, "device %d out of range [0, %d)", device, count);
    const RcclApi &a = rccl();
    if (!a.error.empty()) return fail(SDRG_E_UNSUPPORTED, "%s", a.error.c_str());
    DeviceScope dscope(device);  // the communicator binds to the current device
    if (dscope.error() != hipSuccess) return fail(SDRG_E_HIP, "hipSetDevice(%d) failed", device);
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    sdrg_dist *d = new sdrg_dist();
    ncclResult_t r = a.comm_init_rank(&d->comm, world_size, u, rank);
    if (r != ncclSuccess) {
        delete d;
        return rccl_fail(a, r, "ncclCommInitRank");
    }
    d->rank = rank;
    d->rccl_data = world_size > 1;
    d->world = world_size;
    d->device = device;
    *out = d;
    return SDRG_OK;
}

int32_t sdrg_dist_destroy(sdrg_dist *d) {
    if (!d) return SDRG_OK;
    const RcclApi &a = rccl();
    DeviceScope dscope(d->device);
    ncclResult_t r = d->comm && a.comm_destroy ? a.comm_destroy(d->comm) : ncclSuccess;
    delete d;
    if (r != ncclSuccess) return rccl_fail(a, r, "ncclCommDestroy");
    return SDRG_OK;
}

int32_t sdrg_dist_info(const sdrg_dist *d, int32_t *rank, int32_t *world_size, int32_t *rccl_version,
                       int32_t *rccl_data) {
    if (!d) return fail(SDRG_E_INVALID, "null dist");
    if (rccl_data) *rccl_data = d->rccl_data ? 1 : 0;
    if (rank) *rank = d->rank;
    if (world_size) *world_size = d->world;
    if (rccl_version) {
        int v = 0;
        const RcclApi &a = rccl();
        if (a.get_version) (void)a.get_version(&v);
        *rccl_version = v;
    }
    return SDRG_OK;
}

int32_t sdrg_dist_set_one_rank_rccl(sdrg_dist *d, int32_t on) {
    if (!d) return fail(SDRG_E_INVALID, "null dist");
    d->rccl_data = d->world > 1 || on != 0;
    return SDRG_OK;
}

int32_t sdrg_device_alloc(int32_t device, size_t bytes, void **out) {
    if (!out) return fail(SDRG_E_INVALID, "null out");
    *out = nullptr;
    if (bytes == 0) return fail(SDRG_E_INVALID, "zero-byte device allocation");
    if (const int32_t rc = check_device(device)) return rc;
    DeviceScope dscope(device);
    if (dscope.error() != hipSuccess) return fail(SDRG_E_HIP, "hipSetDevice(%d) failed", device);
    if (hipMalloc(out, bytes) != hipSuccess) {
        *out = nullptr;
        return fail(SDRG_E_NOMEM, "hipMalloc of %zu bytes on device %d failed", bytes, device);
    }
    return SDRG_OK;
}

int32_t sdrg_device_free(int32_t device, void *p) {
    if (!p) return SDRG_OK;
    if (const int32_t rc = check_device(device)) return rc;
    DeviceScope dscope(device);
    if (dscope.error() != hipSuccess) return fail(SDRG_E_HIP, "hipSetDevice(%d) failed", device);
    if (hipFree(p) != hipSuccess) return fail(SDRG_E_HIP, "hipFree failed");
    return SDRG_OK;
}

int32_t sdrg_measure_hbm_copy(int32_t device, size_t bytes, int32_t reps, double *gbs) {
    if (!gbs) return fail(SDRG_E_INVALID, "null gbs");
    *gbs = 0.0;
    if (bytes < 16 || reps <= 0) return fail(SDRG_E_INVALID, "bytes %zu / reps %d", bytes, reps);
    if (const int32_t rc = check_device(device)) return rc;
    DeviceScope dscope(device);
    if (dscope.error() != hipSuccess) return fail(SDRG_E_HIP, "hipSetDevice(%d) failed", device);
    const hipError_t e = sdrg::measure_stream_copy(bytes, reps, gbs);
    if (e != hipSuccess) return fail(SDRG_E_HIP, "stream copy probe: %s", hipGetErrorString(e));
    return SDRG_OK;
}

int32_t sdrg_memcpy(int32_t device, void *dst, const void *src, size_t bytes) {
    if ((!dst || !src) && bytes) return fail(SDRG_E_INVALID, "null buffer");
    if (!bytes) return SDRG_OK;
    if (const int32_t rc = check_device(device)) return rc;
    DeviceScope dscope(device);
    if (dscope.error() != hipSuccess) return fail(SDRG_E_HIP, "hipSetDevice(%d) failed", device);
    hipError_t e = hipMemcpy(dst, src, bytes, hipMemcpyDefault);  // synchronous with respect to the host
    if (e != hipSuccess) return fail(SDRG_E_HIP, "hipMemcpy: %s", hipGetErrorString(e));
    return SDRG_OK;
}

}  // extern "C"

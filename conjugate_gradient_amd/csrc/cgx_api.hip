// cgx_api.hip -- the C ABI of include/cgx.h: errors and devices, and the
// kernel-level entry points; the rest of the ABI lives in cgx_setup.hip,
// cgx_exchange.hip and cgx_iterate.hip (shared types: cgx_ctx.h).
#include "cgx_ctx.h"

namespace cgxh {

thread_local char g_err[1024] = "";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

void debug_log(const char *fmt, ...) {
    static const bool on = [] {
        const char *e = std::getenv("CGX_DEBUG");
        return e && *e == '1';
    }();
    if (!on) return;
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    fprintf(stderr, "[cgx] %s\n", buf);
    fflush(stderr);
}

// Per-device workspace for the kernel-level entry points.
std::mutex g_ws_mu;
RedWs g_ws[64];
int dev_ws(RedWs *out) {
    int dev = 0;
    HIPT(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return fail(CGX_ERR_ARG, "device id %d out of range", dev);
    std::lock_guard<std::mutex> lk(g_ws_mu);
    if (!g_ws[dev].partials) {  // both buffers, or neither (a failed call leaves nothing half-made)
        RedWs w{nullptr, nullptr};
        hipError_t e = hipMalloc(&w.partials, kMaxRedBlocks * sizeof(double));
        if (e == hipSuccess) e = hipMalloc(&w.tickets, kTickets * sizeof(unsigned));
        if (e == hipSuccess) e = hipMemset(w.tickets, 0, kTickets * sizeof(unsigned));
        if (e != hipSuccess) {
            if (w.partials) (void)hipFree(w.partials);
            if (w.tickets) (void)hipFree(w.tickets);
            return fail(CGX_ERR_NOMEM, "reduction workspace on device %d: %s", dev, hipGetErrorString(e));
        }
        g_ws[dev] = w;
    }
    *out = g_ws[dev];
    return CGX_OK;
}

int check_dtype(int dtype) {
    if (dtype != CGX_F64 && dtype != CGX_F32_REF) return fail(CGX_ERR_ARG, "dtype must be CGX_F64 or CGX_F32_REF");
    return CGX_OK;
}

}  // namespace cgxh

extern "C" {

const char *cgx_strerror(int code) {
    switch (code) {
        case CGX_OK: return "ok";
        case CGX_ERR_ARG: return "invalid argument";
        case CGX_ERR_HIP: return "HIP runtime error";
        case CGX_ERR_RCCL: return "RCCL error";
        case CGX_ERR_SHAPE: return "shape error";
        case CGX_ERR_NOMEM: return "out of memory";
        case CGX_ERR_STATE: return "call out of order";
        case CGX_ERR_NODEV: return "no GPU device";
        default: return "unknown error";
    }
}

const char *cgx_last_error(void) { return g_err; }
int cgx_version(void) { return CGX_VERSION; }

int cgx_device_count(int *count) {
    if (!count) return fail(CGX_ERR_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return CGX_OK;
}

int cgx_hip_last_error(void) { return (int)hipPeekAtLastError(); }

int cgx_device_pci_bus_id(int device, char *buf, int len) {
    if (!buf || len < 13) return fail(CGX_ERR_ARG, "buf is NULL or shorter than 13 bytes");
    HIPT(hipDeviceGetPCIBusId(buf, len, device));
    return CGX_OK;
}

int cgx_device_link(int device_a, int device_b, int *link_type, int *hops, int *peer) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(CGX_ERR_NODEV, "no HIP device visible");
    if (device_a < 0 || device_a >= n || device_b < 0 || device_b >= n)
        return fail(CGX_ERR_ARG, "devices %d, %d: %d visible", device_a, device_b, n);
    if (link_type) *link_type = -1;
    if (hops) *hops = -1;
    if (peer) *peer = 0;
    if (device_a == device_b) return CGX_OK;
    uint32_t lt = 0, hc = 0;
    if (hipExtGetLinkTypeAndHopCount(device_a, device_b, &lt, &hc) == hipSuccess) {
        if (link_type) *link_type = (int)lt;
        if (hops) *hops = (int)hc;
    }
    (void)hipGetLastError();  // a device pair HIP cannot describe is not an error of the caller's next call
    int can = 0;
    HIPT(hipDeviceCanAccessPeer(&can, device_a, device_b));
    if (peer) *peer = can;
    return CGX_OK;
}

// ---- kernel-level entry points ---------------------------------------------------------
int cgx_dev_malloc(void **ptr, size_t bytes) {
    if (!ptr) return fail(CGX_ERR_ARG, "ptr is NULL");
    hipError_t e = hipMalloc(ptr, bytes ? bytes : 16);
    if (e != hipSuccess) return fail(CGX_ERR_NOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    return CGX_OK;
}
int cgx_dev_free(void *ptr) {
    if (ptr) HIPT(hipFree(ptr));
    return CGX_OK;
}
int cgx_memcpy_h2d(void *dst, const void *src, size_t bytes) {
    HIPT(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return CGX_OK;
}
int cgx_memcpy_d2h(void *dst, const void *src, size_t bytes) {
    HIPT(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return CGX_OK;
}
int cgx_dev_synchronize(void) {
    HIPT(hipDeviceSynchronize());
    return CGX_OK;
}

int cgx_matvec(int dtype, const void *A, int64_t lda, int64_t rows, int64_t cols, const void *v, void *out,
               void *stream) {
    TRY(check_dtype(dtype));
    if (rows < 0 || cols < 0 || lda < cols) return fail(CGX_ERR_SHAPE, "bad matVec shape");
    if (!A || !v || !out) return fail(CGX_ERR_ARG, "NULL pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (dtype == CGX_F32_REF) {
        HIPT(matvec_ref_f32(static_cast<const float *>(A), lda, rows, cols, static_cast<const float *>(v),
                            static_cast<float *>(out), s));
        return CGX_OK;
    }
    int dev = 0;
    HIPT(hipGetDevice(&dev));
    RedWs ws;
    TRY(dev_ws(&ws));
    MatvecPlan pl = plan_matvec_f64(dev, rows, 0, 0, -1, 0, cols);
    const char *sm = std::getenv("CGX_MV_SMALL");
    if (cols == lda && sm && *sm == '2') {  // the solver's LDS-staged kernel here too (tests)
        const MatvecPlan sp = plan_matvec_small_f64(dev, rows, lda);
        if (sp.small) pl = sp;
    }
    HIPT(matvec_f64(pl, static_cast<const double *>(A), lda, rows, cols, static_cast<const double *>(v),
                    static_cast<double *>(out), nullptr, nullptr, ws, s));
    return CGX_OK;
}

int cgx_dot(int dtype, int64_t n, const void *a, const void *b, void *out_dev, void *stream) {
    TRY(check_dtype(dtype));
    if (!a || !b || !out_dev || n < 0) return fail(CGX_ERR_ARG, "bad argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (dtype == CGX_F32_REF) {
        HIPT(dot_ref_f32(n, static_cast<const float *>(a), static_cast<const float *>(b), static_cast<float *>(out_dev), s));
        return CGX_OK;
    }
    RedWs ws;
    TRY(dev_ws(&ws));
    HIPT(dot_f64(n, static_cast<const double *>(a), static_cast<const double *>(b), static_cast<double *>(out_dev), ws, s));
    return CGX_OK;
}

int cgx_residual(int dtype, int64_t n, const void *b, const void *Ax, void *r, void *p, void *rr_dev,
                 void *stream) {
    TRY(check_dtype(dtype));
    if (!b || !Ax || !r || !p || n < 0) return fail(CGX_ERR_ARG, "bad argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (dtype == CGX_F32_REF) {
        HIPT(residual_ref_f32(n, static_cast<const float *>(b), static_cast<const float *>(Ax), static_cast<float *>(r),
                              static_cast<float *>(p), s));
        if (rr_dev)
            HIPT(dot_ref_f32(n, static_cast<const float *>(r), static_cast<const float *>(r), static_cast<float *>(rr_dev), s));
        return CGX_OK;
    }
    RedWs ws;
    TRY(dev_ws(&ws));
    HIPT(residual_f64(n, static_cast<const double *>(b), static_cast<const double *>(Ax), static_cast<double *>(r),
                      static_cast<double *>(p), static_cast<double *>(rr_dev), ws, s));
    return CGX_OK;
}

int cgx_update_xr(int dtype, int64_t n, void *x, void *r, const void *p, const void *Ap, const void *rsold_dev,
                  const void *pAp_dev, void *rr_dev, void *stream) {
    TRY(check_dtype(dtype));
    if (!x || !r || !p || !Ap || !rsold_dev || !pAp_dev || !rr_dev || n < 0) return fail(CGX_ERR_ARG, "bad argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (dtype == CGX_F32_REF) {
        HIPT(update_xr_ref_f32(n, static_cast<float *>(x), static_cast<float *>(r), static_cast<const float *>(p),
                               static_cast<const float *>(Ap), static_cast<const float *>(rsold_dev),
                               static_cast<const float *>(pAp_dev), s));
        HIPT(dot_ref_f32(n, static_cast<const float *>(r), static_cast<const float *>(r), static_cast<float *>(rr_dev), s));
        return CGX_OK;
    }
    RedWs ws;
    TRY(dev_ws(&ws));
    HIPT(update_xr_f64(n, static_cast<double *>(x), static_cast<double *>(r), static_cast<const double *>(p),
                       static_cast<const double *>(Ap), static_cast<const double *>(rsold_dev),
                       static_cast<const double *>(pAp_dev), static_cast<double *>(rr_dev), ws, s));
    return CGX_OK;
}

int cgx_update_p(int dtype, int64_t n, void *p, const void *r, const void *rr_dev, const void *rsold_dev,
                 void *stream) {
    TRY(check_dtype(dtype));
    if (!p || !r || !rr_dev || !rsold_dev || n < 0) return fail(CGX_ERR_ARG, "bad argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (dtype == CGX_F32_REF)
        HIPT(update_p_ref_f32(n, static_cast<float *>(p), static_cast<const float *>(r), static_cast<const float *>(rr_dev),
                              static_cast<const float *>(rsold_dev), s));
    else
        HIPT(update_p_f64(n, static_cast<double *>(p), static_cast<const double *>(r), static_cast<const double *>(rr_dev),
                          static_cast<const double *>(rsold_dev), s));
    return CGX_OK;
}

int cgx_conjugrad(const void *A, const void *b, void *x, int64_t n, int flags, double eps, int64_t max_iter,
                  cgx_stats *st) {
    if (!A || !b || !x) return fail(CGX_ERR_ARG, "cgx_conjugrad: A, b and x are required");
    cgx_ctx *ctx = nullptr;
    int rc = cgx_create(&ctx, n, 0, flags);
    if (rc != CGX_OK) return rc;
    rc = cgx_set_system(ctx, A, b, x);
    if (rc == CGX_OK) rc = cgx_solve(ctx, x, eps, max_iter, st);
    if (rc != CGX_OK) {  // keep the first failure's detail over the teardown's
        std::string keep = g_err;
        (void)cgx_destroy(ctx);
        snprintf(g_err, sizeof g_err, "%s", keep.c_str());
        return rc;
    }
    return cgx_destroy(ctx);
}

}  // extern "C"

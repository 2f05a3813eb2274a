/*
 * pcr_api.h -- C ABI of libpcr.so, the MI355X (gfx950) registration core.
 *
 * Plain pointers + sizes, no torch types.  Every pointer argument named as a
 * device buffer must be device (HBM) memory of the current HIP device; outputs
 * are caller-allocated (the reference's ownership rule,
 * dip/torch-nndistance/torch_nndistance/__init__.py:17-20,42-43).  Work is
 * enqueued on `stream` (a hipStream_t; NULL = legacy default stream, which is
 * what the reference launcher uses, nnd_cuda.cu:152-153) and is asynchronous
 * unless stated otherwise.
 *
 * Return value: PCR_OK (0) or a negative PCR_ERR_* code; pcr_last_error()
 * returns a thread-local message for the last failure.  (The reference CUDA
 * launcher prints and returns 0 / 1, nnd_cuda.cu:155-161; the Python layer
 * maps PCR_OK -> 1 and raises on failure.)
 */
#ifndef PCR_API_H
#define PCR_API_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCR_OK 0
#define PCR_ERR_ARG (-1)
#define PCR_ERR_HIP (-2)
#define PCR_ERR_NOMEM (-3)

typedef void *pcr_stream_t; /* hipStream_t */

const char *pcr_last_error(void);
int pcr_version(void);

/* ---------------------------------------------------------------------------
 * a1 -- brute-force bidirectional 1-NN ("nnd" / Chamfer building block).
 * Replaces nnd_forward_cuda (dip/torch-nndistance/src/my_lib_cuda.cpp:25-41)
 * -> NmDistanceKernelLauncher (nnd_cuda.cu:132-162).
 *   xyz1 (b,n,3) f32, xyz2 (b,m,3) f32, contiguous AoS, device.
 *   dist1 (b,n) f32 / idx1 (b,n) i32: for each xyz1 point, min over xyz2 of
 *   (dx*dx+dy*dy)+dz*dz in f32 (no FMA) and the FIRST index attaining it;
 *   dist2/idx2 the same from xyz2 to xyz1.  Bit-exact with my_lib.cpp:3-25.
 *   m == 0 (resp. n == 0) yields dist 0, idx 0 (my_lib.cpp seed values).
 * ------------------------------------------------------------------------- */
int pcr_nnd_forward(const float *xyz1, const float *xyz2, int32_t b, int32_t n, int32_t m,
                    float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                    pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * a2 -- gradient of (dist1, dist2) w.r.t. (xyz1, xyz2).
 * Replaces nnd_backward_cuda (my_lib_cuda.cpp:44-72) -> NmDistanceGradKernel
 * (nnd_cuda.cu:164-222).  gxyz1 (b,n,3), gxyz2 (b,m,3) are fully written (the
 * caller need not zero them).  Deterministic: the scatter terms are summed in
 * the exact order of the reference CPU loop (my_lib.cpp:93-130), so the result
 * is bitwise reproducible and bit-identical to the CPU reference (the CUDA
 * reference uses float atomics and is not).
 * ------------------------------------------------------------------------- */
int pcr_nnd_backward(const float *xyz1, const float *xyz2, const float *graddist1,
                     const float *graddist2, const int32_t *idx1, const int32_t *idx2,
                     int32_t b, int32_t n, int32_t m, float *gradxyz1, float *gradxyz2,
                     pcr_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PCR_API_H */

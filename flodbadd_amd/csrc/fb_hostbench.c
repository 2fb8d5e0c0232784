/* fb_hostbench.c -- bench.py's per-frame producer loop (not the product): the reference's reader
 * thread hands over ONE frame per next_packet() (src/capture.rs:1088-1092), so the ring's per-frame
 * entry point is timed from native code, one call per frame, the way a Rust capture loop calls it
 * (a Python loop would time the interpreter).  The entry point is passed as a function pointer
 * (the library's fb_ring_push), so this file links against nothing. */
#include <stdint.h>
#include <time.h>

typedef int (*push_fn)(void* ring, const uint8_t* frame, uint32_t caplen);

/* Push frames [0, n) of the packed batch `reps` times, one call per frame; returns 0 or the first
 * non-zero return code; *seconds = wall time of the loop (CLOCK_MONOTONIC). */
int fb_hostbench_push_frames(void* fn, void* ring, const uint8_t* frames, const uint32_t* offsets, uint32_t n,
                             uint32_t reps, double* seconds) {
    push_fn push = (push_fn)fn;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint32_t r = 0; r < reps; ++r)
        for (uint32_t k = 0; k < n; ++k) {
            const int rc = push(ring, frames + offsets[k], offsets[k + 1] - offsets[k]);
            if (rc) return rc;
        }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    return 0;
}

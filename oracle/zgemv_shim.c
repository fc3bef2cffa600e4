/* TEST INFRASTRUCTURE ONLY. Symbol alias so the reference Fortran (which calls the BLAS name
 * `zgemv_`) links against the image's OpenBLAS, which scipy ships with the `scipy_` prefix.
 * No arithmetic here: every argument (including Fortran's hidden CHARACTER length) is forwarded. */
#include <stddef.h>
extern void scipy_zgemv_(const char*, const int*, const int*, const void*, const void*, const int*,
                         const void*, const int*, const void*, void*, const int*, size_t);
void zgemv_(const char* t, const int* m, const int* n, const void* a, const void* A, const int* lda,
            const void* x, const int* incx, const void* b, void* y, const int* incy, size_t tl) {
    scipy_zgemv_(t, m, n, a, A, lda, x, incx, b, y, incy, tl);
}

// pageable_copy_probe: how the HIP runtime carries hipMemcpyAsync between
// pageable host memory and the device, by source/destination alignment and
// size (round 5: the GPU faults of two suite runs sat at a staged H2D whose
// pageable source was 2-byte aligned).  Run under
// `rocprofv3 --kernel-trace --memory-copy-trace`: a copy the runtime does with
// a blit shader shows up as a kernel, an SDMA copy as a memory copy.  Plain
// malloc'ed buffers, every copy in bounds: nothing here reads outside them.
//   pageable_copy_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main() {
    const size_t sizes[] = {1572874, 1572880, 3145748, 6291466, 33554432};
    const size_t shifts[] = {0, 2, 4, 16};
    const size_t cap = (64u << 20) + 4096;
    char* h = static_cast<char*>(malloc(cap));
    char* h2 = static_cast<char*>(malloc(cap));
    memset(h, 1, cap);
    memset(h2, 0, cap);
    void* d = nullptr;
    CK(hipMalloc(&d, cap));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int dir = 0; dir < 2; dir++)
        for (size_t n : sizes)
            for (size_t sh : shifts) {
                char* hp = (dir ? h2 : h) + 64 + sh;  // malloc'ed: 16-byte aligned base
                for (int rep = 0; rep < 3; rep++) {
                    const auto t0 = std::chrono::steady_clock::now();
                    if (dir == 0) CK(hipMemcpyAsync(d, hp, n, hipMemcpyHostToDevice, s));
                    else CK(hipMemcpyAsync(hp, d, n, hipMemcpyDeviceToHost, s));
                    CK(hipStreamSynchronize(s));
                    const double us =
                        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                    if (rep == 2)
                        printf("{\"dir\": \"%s\", \"bytes\": %zu, \"host_mod16\": %zu, \"us\": %.1f, \"GBps\": %.2f}\n",
                               dir ? "d2h" : "h2d", n, (size_t)((uintptr_t)hp % 16), us, n / us / 1e3);
                }
            }
    CK(hipFree(d));
    free(h);
    free(h2);
    return 0;
}

// PCIe transfer options for the host-buffer API (fa2_*_host): pageable hipMemcpy,
// hipHostRegister of the caller's buffer (+ copy + unregister), and a pre-pinned
// buffer, H2D and D2H, per size.  Prints GB/s of each (wall, including registration).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));         \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main() {
    const size_t sizes[] = {size_t(32) << 20, size_t(256) << 20};
    for (size_t n : sizes) {
        std::vector<char> host(n);
        std::memset(host.data(), 1, n);
        void* dev = nullptr;
        CK(hipMalloc(&dev, n));
        CK(hipMemcpy(dev, host.data(), n, hipMemcpyHostToDevice));  // warm
        for (int rep = 0; rep < 2; ++rep) {
            double t0 = now();
            CK(hipMemcpy(dev, host.data(), n, hipMemcpyHostToDevice));
            double t1 = now();
            CK(hipMemcpy(host.data(), dev, n, hipMemcpyDeviceToHost));
            double t2 = now();
            CK(hipHostRegister(host.data(), n, hipHostRegisterPortable));
            double t3 = now();
            CK(hipMemcpyAsync(dev, host.data(), n, hipMemcpyHostToDevice, nullptr));
            CK(hipStreamSynchronize(nullptr));
            double t4 = now();
            CK(hipMemcpyAsync(host.data(), dev, n, hipMemcpyDeviceToHost, nullptr));
            CK(hipStreamSynchronize(nullptr));
            double t5 = now();
            CK(hipHostUnregister(host.data()));
            double t6 = now();
            std::printf("%4zu MB: pageable H2D %6.1f GB/s D2H %6.1f | register %6.2f ms (%5.1f GB/s) pinned H2D %6.1f "
                        "D2H %6.1f unregister %6.2f ms\n",
                        n >> 20, n / (t1 - t0) / 1e9, n / (t2 - t1) / 1e9, (t3 - t2) * 1e3, n / (t3 - t2) / 1e9,
                        n / (t4 - t3) / 1e9, n / (t5 - t4) / 1e9, (t6 - t5) * 1e3);
        }
        void* pin = nullptr;
        CK(hipHostMalloc(&pin, n, hipHostMallocDefault));
        std::memset(pin, 1, n);
        double t0 = now();
        CK(hipMemcpy(dev, pin, n, hipMemcpyHostToDevice));
        double t1 = now();
        CK(hipMemcpy(pin, dev, n, hipMemcpyDeviceToHost));
        double t2 = now();
        double t3 = now();
        std::memcpy(pin, host.data(), n);
        double t4 = now();
        std::printf("%4zu MB: hipHostMalloc buffer H2D %6.1f GB/s D2H %6.1f; host memcpy into it %6.1f GB/s\n", n >> 20,
                    n / (t1 - t0) / 1e9, n / (t2 - t1) / 1e9, n / (t4 - t3) / 1e9);
        CK(hipHostFree(pin));
        CK(hipFree(dev));
    }
    return 0;
}

// tools/micro/init_par.cpp — HIP start-up steps of a fresh process, serial or overlapped:
//   ./init_par serial|parallel|nosecond
// runtime start (hipGetDeviceCount), the main stream, and the staging set (a second stream,
// 4 x 8 MB pinned buffers, one 1 MB copy each way), the staging set run either after the
// main stream or on a second thread beside it.  Prints one line of step times (ms).
// Build: hipcc -O2 init_par.cpp -o init_par
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b)
{
    return std::chrono::duration<double, std::milli>(b - a).count();
}

int main(int argc, char **argv)
{
    const char *mode = argc > 1 ? argv[1] : "serial";
    const auto t0 = clk::now();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return 1;
    const auto t1 = clk::now();
    hipStream_t s0 = nullptr, s1 = nullptr;
    void *ring[4] = {};
    void *d = nullptr;
    double t_main = 0, t_stage = 0;
    auto main_stream = [&] {
        const auto a = clk::now();
        (void)hipSetDevice(0);
        (void)hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
        t_main = ms(a, clk::now());
    };
    auto staging = [&] {
        const auto a = clk::now();
        (void)hipSetDevice(0);
        if (strcmp(mode, "nosecond") != 0) (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
        for (auto &r : ring) (void)hipHostMalloc(&r, 8u << 20, hipHostMallocDefault);
        (void)hipMalloc(&d, 1u << 20);
        hipStream_t s = s1 ? s1 : s0;
        (void)hipMemcpyAsync(d, ring[0], 1u << 20, hipMemcpyHostToDevice, s);
        (void)hipMemcpyAsync(ring[1], d, 1u << 20, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        t_stage = ms(a, clk::now());
    };
    if (strcmp(mode, "parallel") == 0) {
        std::thread th(staging);
        main_stream();
        th.join();
    } else {
        main_stream();
        staging();
    }
    const auto t2 = clk::now();
    printf("%s runtime %.1f main_stream %.1f staging %.1f after_runtime %.1f total %.1f\n", mode,
           ms(t0, t1), t_main, t_stage, ms(t1, t2), ms(t0, t2));
    return 0;
}

// tools/micro/write_rate.cpp — how fast can `fpmash dist` put its text into a regular file?
// Writes SIZE bytes of a pre-made buffer to PATH by: (1) one pwrite stream, (2) T threads
// pwriting disjoint pieces, (3) T threads copying into a MAP_SHARED mapping after one
// ftruncate, (4) the same with MADV_POPULATE_WRITE per piece, (5) fallocate + T pwrite threads,
// (6) fallocate alone, (7) one pwrite stream into the allocated pages and (8)/(9) T threads
// writing through a shared mapping of allocated pages.
// Build: g++ -O2 -pthread tools/micro/write_rate.cpp -o /tmp/write_rate
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv)
{
    const char *path = argc > 1 ? argv[1] : "/dev/shm/fpm_write_rate";
    const size_t size = (argc > 2 ? strtoull(argv[2], nullptr, 10) : 2048) << 20;
    const int T = argc > 3 ? atoi(argv[3]) : 8;
    const size_t piece = 40u << 20;
    std::vector<char> src(piece);
    for (size_t i = 0; i < piece; i++) src[i] = "ACGT\t1/\n"[i & 7];
    auto run = [&](const char *name, auto body) {
        unlink(path);
        int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
        const double t0 = now();
        body(fd);
        const double t1 = now();
        close(fd);
        unlink(path);
        printf("%-28s %7.1f ms  %6.2f GB/s\n", name, (t1 - t0) * 1e3, size / (t1 - t0) / 1e9);
    };
    const size_t np = (size + piece - 1) / piece;
    auto par = [&](auto fn) {
        std::atomic<size_t> next{0};
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&] {
                for (size_t p; (p = next.fetch_add(1)) < np;) fn(p * piece, std::min(piece, size - p * piece));
            });
        for (auto &x : th) x.join();
    };
    run("pwrite, 1 thread", [&](int fd) {
        for (size_t p = 0; p < np; p++)
            if (pwrite(fd, src.data(), std::min(piece, size - p * piece), p * piece) < 0) abort();
    });
    run("pwrite, T threads", [&](int fd) {
        par([&](size_t at, size_t n) { if (pwrite(fd, src.data(), n, at) < 0) abort(); });
    });
    for (int pop = 0; pop < 2; pop++)
        run(pop ? "mmap + populate, T threads" : "mmap, T threads", [&](int fd) {
            if (ftruncate(fd, size)) abort();
            char *m = (char *)mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            if (m == MAP_FAILED) abort();
            par([&](size_t at, size_t n) {
                if (pop) madvise(m + at, n, 23);
                memcpy(m + at, src.data(), n);
            });
            munmap(m, size);
        });
    run("fallocate + mmap, T threads", [&](int fd) {
        if (fallocate(fd, 0, 0, size)) perror("fallocate");
        char *m = (char *)mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (m == MAP_FAILED) abort();
        par([&](size_t at, size_t n) { madvise(m + at, n, 23); memcpy(m + at, src.data(), n); });
        munmap(m, size);
    });
    run("fallocate + pwrite T thr", [&](int fd) {
        if (fallocate(fd, 0, 0, size)) perror("fallocate");
        par([&](size_t at, size_t n) { if (pwrite(fd, src.data(), n, at) < 0) abort(); });
    });
    // (6) / (7): the two halves of (5) timed apart — the pages allocated ahead (what the CLI
    // could do while the HIP runtime starts), then one pwrite stream into them
    {
        unlink(path);
        int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
        double t0 = now();
        if (fallocate(fd, 0, 0, size)) perror("fallocate");
        double t1 = now();
        printf("%-28s %7.1f ms  %6.2f GB/s\n", "fallocate alone", (t1 - t0) * 1e3, size / (t1 - t0) / 1e9);
        t0 = now();
        for (size_t p = 0; p < np; p++)
            if (pwrite(fd, src.data(), std::min(piece, size - p * piece), p * piece) < 0) abort();
        t1 = now();
        printf("%-28s %7.1f ms  %6.2f GB/s\n", "pwrite 1 thr, pages allocated", (t1 - t0) * 1e3, size / (t1 - t0) / 1e9);
        close(fd);
        unlink(path);
    }
    // (8) / (9): pages allocated ahead (untimed), then T threads writing into a shared mapping
    // of them (with / without MADV_POPULATE_WRITE per piece), munmap included
    for (int pop = 0; pop < 2; pop++) {
        unlink(path);
        int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
        if (fallocate(fd, 0, 0, size)) perror("fallocate");
        double t0 = now();
        char *m = (char *)mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (m == MAP_FAILED) abort();
        par([&](size_t at, size_t n) { if (pop) madvise(m + at, n, 23); memcpy(m + at, src.data(), n); });
        double t1 = now();
        munmap(m, size);
        double t2 = now();
        printf("%-28s %7.1f ms  %6.2f GB/s  (munmap %.1f ms)\n", pop ? "alloc'd, mmap+populate T thr" : "alloc'd, mmap T thr",
               (t2 - t0) * 1e3, size / (t2 - t0) / 1e9, (t2 - t1) * 1e3);
        close(fd);
        unlink(path);
    }
    return 0;
}

// registry_stress.cpp — the declared host ranges of libmi_reduce
// (mi_host_declare / mi_host_undeclare / classification) under concurrent
// readers and writers, for the host sanitizers (tests/test_registry_sanitizers.py
// builds it against ASan and TSan builds of the library's host code).
// Readers: threads that classify operands inside a range held declared for
// the whole run (must always see kind 2, pageable), and short-lived reader
// threads (slot recycling).  Writers: threads that declare and undeclare
// ranges of their own in a loop (snapshot publication + grace periods).
// Exiting readers: threads whose last read happens inside a thread_local
// destructor that runs after the library has released the thread's reader
// slot: that read must take the locked path, not a slot another
// thread may own.
// Exit 0 when every check held.  No GPU is needed: undeclared pointers are
// classified by HIP, which reports pageable (or no device) on a CPU host.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/mi_reduce.h"

// Constructed before the thread's first classification, so destroyed after
// the library's own thread_local slot reference: its read is a late one.
struct LateReader {
    const unsigned char* p = nullptr;
    std::atomic<long>* bad = nullptr;
    ~LateReader() {
        if (p && mi_host_declared_kind(p, 64) != 2) (*bad)++;
    }
};
thread_local LateReader t_late;

int main(int argc, char** argv) {
    const double seconds = argc > 1 ? atof(argv[1]) : 1.0;
    std::vector<unsigned char> held(1 << 20);
    if (mi_host_declare(held.data(), held.size()) != 0) {
        fprintf(stderr, "declare failed: %s\n", mi_last_error());
        return 1;
    }
    std::atomic<bool> stop{false};
    std::atomic<long> bad{0}, reads{0}, cycles{0};
    auto reader = [&](int seed) {
        size_t i = (size_t)seed * 977;
        while (!stop.load(std::memory_order_relaxed)) {
            const size_t off = (i * 4099) % (held.size() - 256);
            int dev = -1;
            if (mi_host_declared_kind(held.data() + off, 256) != 2) bad++;
            if (mi_pointer_kind_range(held.data() + off, 64, &dev) != 2) bad++;
            reads++;
            i++;
        }
    };
    auto writer = [&](int seed) {
        std::vector<std::vector<unsigned char>> mine(16, std::vector<unsigned char>(4096 + 64 * seed));
        while (!stop.load(std::memory_order_relaxed)) {
            for (auto& b : mine)
                if (mi_host_declare(b.data(), b.size()) != 0) bad++;
            for (auto& b : mine)
                if (mi_host_declared_kind(b.data() + 1, 16) != 2) bad++;
            for (auto& b : mine)
                if (mi_host_undeclare(b.data()) != 0) bad++;
            cycles++;
        }
    };
    std::vector<std::thread> ts;
    for (int r = 0; r < 6; r++) ts.emplace_back(reader, r);
    for (int w = 0; w < 2; w++) ts.emplace_back(writer, w);
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
        std::vector<std::thread> shortlived;  // take a reader slot, read, exit: the slot comes back
        for (int r = 0; r < 8; r++)
            shortlived.emplace_back([&, r] {
                if (r % 2) {  // a read at thread exit too, after the slot went back
                    t_late.bad = &bad;
                    t_late.p = held.data() + 256;
                }
                if (mi_host_declared_kind(held.data() + 128, 64) != 2) bad++;
            });
        for (auto& t : shortlived) t.join();
    }
    stop = true;
    for (auto& t : ts) t.join();
    if (mi_host_undeclare(held.data()) != 0) bad++;
    if (mi_host_declared_kind(held.data(), 16) != -1) bad++;
    printf("registry_stress: reads %ld, writer cycles %ld, failures %ld\n", reads.load(), cycles.load(), bad.load());
    return bad.load() == 0 ? 0 : 1;
}

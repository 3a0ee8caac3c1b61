// ThreadSanitizer driver for pe_rowstore.cpp: 8 readers (get + increment)
// race one writer (store_row for the first half of the rows, then one
// 4-thread store_rows bulk fill for the rest) on the same store.  Built and run by
// tests/test_rowstore.py::test_rowstore_under_thread_sanitizer (host code
// only, no device).
#include <atomic>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "shd_pathengine.h"

int main() {
    const int n = 3000, k = 300;
    std::vector<int32_t> att(k);
    for (int j = 0; j < k; ++j) att[j] = 7 * j + 3;
    ShdRowStore* st = nullptr;
    if (shd_rowstore_new(n, att.data(), k, &st)) return 2;
    std::atomic<bool> stop{false};
    std::atomic<long> bad{0}, incs{0};
    std::vector<std::thread> th;
    for (int i = 0; i < 8; ++i)
        th.emplace_back([&, i] {
            std::mt19937 r(i);
            while (!stop.load()) {
                const int a = r() % k, b = r() % k;
                double lat, rel;
                if (shd_rowstore_get(st, att[a], att[b], &lat, &rel, nullptr, nullptr)) {
                    const int lo = a < b ? a : b, hi = a < b ? b : a;
                    if (lat != 1000.0 * lo + hi) bad++;
                    if (shd_rowstore_increment(st, att[a], att[b]) == 0) incs++;
                }
            }
        });
    std::vector<double> lat(k), rel(k, 0.5);
    std::vector<uint8_t> fl(k, 0);
    const int half = k / 2;
    for (int a = 0; a < half; ++a) {
        for (int b = 0; b < k; ++b) lat[b] = a <= b ? 1000.0 * a + b : 1000.0 * b + a;
        if (shd_rowstore_store_row(st, att[a], lat.data(), rel.data(), fl.data(), 0, nullptr) < 0)
            return 3;
    }
    {
        const int cnt = k - half;
        std::vector<int32_t> src(cnt);
        std::vector<double> L((size_t)cnt * k), R((size_t)cnt * k, 0.5);
        std::vector<uint8_t> F((size_t)cnt * k, 0);
        for (int i = 0; i < cnt; ++i) {
            const int a = half + i;
            src[i] = att[a];
            for (int b = 0; b < k; ++b) L[(size_t)i * k + b] = a <= b ? 1000.0 * a + b : 1000.0 * b + a;
        }
        if (shd_rowstore_store_rows(st, src.data(), cnt, L.data(), R.data(), F.data(), k, 0, nullptr, 4,
                                    nullptr) < 0)
            return 5;
    }
    stop = true;
    for (auto& t : th) t.join();
    uint64_t total = 0;
    for (int a = 0; a < k; ++a)
        for (int b = a; b < k; ++b) {
            uint64_t pc = 0;
            if (!shd_rowstore_get(st, att[a], att[b], nullptr, nullptr, nullptr, &pc)) return 4;
            total += pc;
        }
    const bool ok = bad == 0 && (long)total == incs && shd_rowstore_size(st) == (int64_t)k * (k + 1) / 2;
    shd_rowstore_free(st);
    std::printf("%s bad=%ld incs=%ld total=%llu\n", ok ? "OK" : "FAIL", bad.load(), incs.load(),
                (unsigned long long)total);
    return ok ? 0 : 1;
}

// tests/maps_host/shim.cpp -- TEST INFRASTRUCTURE ONLY: the pointer classifier of
// quicknet_amd/csrc/qfec_maps.hpp (module/rs.h host-pointer paths) on synthetic
// /proc/self/maps text, for tests/test_maps_classify.py.  Never shipped.
#include "../../quicknet_amd/csrc/qfec_maps.hpp"

extern "C" {
// 1 system memory for certain, 0 ask the runtime, -1 no mapping parsed
int maps_is_host(const char* text, unsigned long long addr) {
    qfec::MapSnap m;
    if (!m.load_text(text)) return -1;
    size_t hint = 0;
    return m.host((uintptr_t)addr, &hint) ? 1 : 0;
}
int maps_count(const char* text) {
    qfec::MapSnap m;
    m.load_text(text);
    return (int)m.r.size();
}
// this process's own maps: 1 if addr is classified as system memory
int maps_self_is_host(unsigned long long addr) {
    qfec::MapSnap m;
    if (!m.load()) return -1;
    size_t hint = 0;
    return m.host((uintptr_t)addr, &hint) ? 1 : 0;
}
}

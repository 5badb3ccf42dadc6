// qfec_maps.hpp -- which caller pointers are system memory, from the process's mappings
// (module/rs.h host-pointer paths, qfec_rs_abi.cpp classify_ptrs).  Header-only so the CPU
// suite can hold the rules to synthetic /proc/self/maps text (tests/test_maps_classify.py).
#pragma once

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

namespace qfec {

// The process's mappings (/proc/self/maps), read once per call, answer for most pointers without
// a runtime probe (one probe per 64 KiB window cost ~14 ms on a 1.3 M-pointer call, r05g).  Device
// memory is CPU-visible only through the GPU driver's files (the render node, /dev/kfd, or a
// dma-buf), and device memory the CPU cannot see sits in address space with no access rights
// (tools/maps_probe.py, profiles/r05g/maps.log: hipMalloc'd tensors of 4 KiB .. 4 GiB lie in
// "rw-s /dev/dri/renderD*" mappings, pinned and pageable host memory in anonymous or heap
// ones).  So a pointer inside a readable anonymous, heap, stack, tmpfs or regular-file mapping is
// system memory the CPU copies can read and write, whatever the runtime knows about it (pinned,
// registered or managed); every other pointer -- a driver mapping, an inaccessible range, or an
// address the snapshot does not cover -- takes the runtime probe.
struct MapSnap {
    struct Range {
        uintptr_t lo, hi;
        bool host;
    };
    std::vector<Range> r;  // ascending, as the kernel lists them
    static bool host_path(const char* path, char perm_r) {
        if (perm_r != 'r') return false;  // inaccessible: possibly device memory the CPU cannot see
        if (!*path || path[0] == '[') return true;  // anonymous, [heap], [stack], ...
        if (!strncmp(path, "/dev/", 5))  // driver files: only shared-anonymous and tmpfs ones are RAM
            return !strncmp(path, "/dev/zero", 9) || !strncmp(path, "/dev/shm/", 9);
        if (!strncmp(path, "anon_inode:", 11) || !strncmp(path, "/dmabuf", 7) || !strncmp(path, "/memfd:", 7))
            return !strncmp(path, "/memfd:", 7);  // memfd is RAM; dma-buf / other inodes may be device
        return path[0] == '/';  // a regular file's page cache
    }
    // one maps line "lo-hi perms offset dev inode [path]" (a line that does not parse is skipped)
    void add_line(char* line) {
        unsigned long lo = 0, hi = 0;
        char perm[8] = {};
        int path_at = 0;
        if (sscanf(line, "%lx-%lx %7s %*s %*s %*s %n", &lo, &hi, perm, &path_at) < 3) return;
        char* path = line + (path_at > 0 ? path_at : (int)strlen(line));
        path[strcspn(path, "\n")] = 0;
        r.push_back(Range{(uintptr_t)lo, (uintptr_t)hi, host_path(path, perm[0])});
    }
    bool load() {
        r.clear();
        FILE* f = fopen("/proc/self/maps", "r");
        if (!f) return false;
        char line[4096];
        while (fgets(line, sizeof line, f)) add_line(line);
        fclose(f);
        return !r.empty();
    }
    // the same from text (tests)
    bool load_text(const char* text) {
        r.clear();
        std::vector<char> line;
        for (const char* p = text; *p;) {
            const char* e = strchr(p, '\n');
            const size_t n = e ? (size_t)(e - p) : strlen(p);
            line.assign(p, p + n);
            line.push_back(0);
            add_line(line.data());
            p += n + (e ? 1 : 0);
        }
        return !r.empty();
    }
    // true: system memory for certain; false: ask the runtime
    bool host(uintptr_t u, size_t* hint) const {
        size_t i = *hint;
        if (i >= r.size() || u < r[i].lo || u >= r[i].hi) {
            auto it = std::upper_bound(r.begin(), r.end(), u, [](uintptr_t x, const Range& g) { return x < g.lo; });
            if (it == r.begin()) return false;
            i = (size_t)(it - r.begin()) - 1;
            if (u >= r[i].hi) return false;
            *hint = i;
        }
        return r[i].host;
    }
};

}  // namespace qfec

// map_fill.cpp — TEST PROGRAM helper: the Go shim's keydir fill
// (db.kd.entries[key] = kdEntry / delete, core/keydir.go:22-49) as a C++
// std::unordered_map<std::string, entry>, a proxy for the Go map the cgo shim
// of INTEGRATION.md §2 fills after the replay.  Keys come from GCK_OPT_KEYS's
// blob (record i's key_len bytes back to back).
#include <chrono>
#include <cstdint>
#include <string>
#include <unordered_map>

#include "gocask_hip.h"

namespace {
struct entry {  // kdEntry (core/keydir.go:3-9): File is the walk index here
    uint32_t file, value_pos, value_size, crc, ts;
};
}  // namespace

// live = 0: every record in walk order, set / unset (the records mode);
// live = 1: one insert per live key (GCK_OPT_LIVE).  Returns ms; *n_live =
// the map's size afterwards.
extern "C" double shim_map_fill(const gck_rec *recs, uint64_t n, const uint8_t *keys, int live, uint64_t *n_live) {
    const auto t0 = std::chrono::steady_clock::now();
    std::unordered_map<std::string, entry> m;
    if (live) m.reserve(n);
    uint64_t off = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const gck_rec &r = recs[i];
        std::string k(reinterpret_cast<const char *>(keys + off), r.key_len);
        off += r.key_len;
        if (r.flags & GCK_F_TOMBSTONE)
            m.erase(k);
        else
            m[std::move(k)] = entry{r.file, r.value_pos, r.value_size, r.crc, r.ts};
    }
    *n_live = m.size();
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

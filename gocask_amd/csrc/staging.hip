// staging.hip — host-to-device copies of data files that are not page-locked
// (row f2 of SURVEY.md §8: the pinned H2D pipeline behind Open).
//
// gck_replay's files reach the device arena on one copy stream.  Memory the
// caller registered (gck_host_register) is copied by the DMA engine directly.
// Anything else -- pageable memory, or files named by path (gck_replay_paths)
// -- goes through this copier: host threads fill page-locked staging buffers
// (memcpy from the caller's memory, or pread from the file, which needs no
// mapping and takes no page faults) and queue each buffer on the copy stream
// as soon as it is full, so the CPU copies, the PCIe transfer and the
// replays of earlier file groups all overlap.  Pinning a whole database
// first (hipHostRegister of every mmap, then unregistering it) costs more
// than the transfer itself: 1.3 s + 0.5-1.3 s against 0.6 s of PCIe for C3
// (DESIGN.md §9b).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <unordered_set>
#include <vector>

#include "gck_internal.h"

namespace gck {

namespace {
// bytes per staging buffer (GCK_STAGE_MIB overrides, for measurements)
uint64_t stage_chunk() {
    static const uint64_t v = [] {
        const char *e = getenv("GCK_STAGE_MIB");
        const int m = e ? atoi(e) : 0;
        return (uint64_t)(m >= 1 && m <= 256 ? m : 32) << 20;  // 8 MiB: 39-46 GB/s, 32 MiB: 53-55 GB/s
    }();
    return v;
}

// Page-locked staging buffers kept for the process, per device: a copier
// takes the buffers it needs from the free list and gives them back when it
// finishes (concurrent copiers -- gck_replay_multi's device threads, several
// Opens -- never share one); gck_replay_release_cache frees the idle ones.
// Allocating 0.5 GiB of pinned memory per Open would cost more than filling it.
struct StagePool {
    std::mutex mu;
    std::vector<std::pair<int, void *>> idle;  // (device, buffer)
} g_stage;

// A staging buffer: plain memory on transparent huge pages, then registered
// (page-locked and mapped for the device) -- 24 ms for 16 x 32 MiB where
// hipHostMalloc took 82-124 ms (tools/setup_xp.cpp on an MI355X box); the
// allocation sits in front of the first file copy of a process's first Open.
// hipHostMalloc when registration fails.
std::unordered_set<void *> g_stage_reg;  // the registered ones (under g_stage.mu)
void *stage_alloc() {
    constexpr size_t kHuge = 2ull << 20;
    const size_t C = (stage_chunk() + kHuge - 1) & ~(kHuge - 1);
    static const bool reg = !getenv("GCK_STAGE_HOSTMALLOC");  // (A/B knob)
    if (void *p = reg ? aligned_alloc(kHuge, C) : nullptr) {
        (void)madvise(p, C, MADV_HUGEPAGE);
        if (hipHostRegister(p, C, hipHostRegisterDefault) == hipSuccess) {
            g_stage_reg.insert(p);
            return p;
        }
        (void)hipGetLastError();
        free(p);
    }
    void *q = nullptr;
    return hipHostMalloc(&q, stage_chunk(), hipHostMallocDefault) == hipSuccess ? q : nullptr;
}
void stage_free(void *p) {
    if (g_stage_reg.erase(p)) {
        (void)hipHostUnregister(p);
        free(p);
    } else {
        (void)hipHostFree(p);
    }
}

int stage_take(int dev, size_t n, std::vector<void *> &out) {
    std::lock_guard<std::mutex> lk(g_stage.mu);
    for (size_t i = 0; i < g_stage.idle.size() && out.size() < n;)
        if (g_stage.idle[i].first == dev) {
            out.push_back(g_stage.idle[i].second);
            g_stage.idle.erase(g_stage.idle.begin() + (ptrdiff_t)i);
        } else {
            ++i;
        }
    while (out.size() < n) {
        void *q = stage_alloc();
        if (!q) return GCK_ENOMEM;
        out.push_back(q);
    }
    return GCK_OK;
}

void stage_give(int dev, std::vector<void *> &bufs) {
    std::lock_guard<std::mutex> lk(g_stage.mu);
    for (void *q : bufs) g_stage.idle.emplace_back(dev, q);
    bufs.clear();
}

uint32_t copy_threads() {
    if (const char *e = getenv("GCK_COPY_THREADS")) {
        const int v = atoi(e);
        if (v >= 1 && v <= 64) return (uint32_t)v;
    }
    const uint32_t hw = std::thread::hardware_concurrency();
    return std::max<uint32_t>(2, std::min<uint32_t>(8, hw ? hw / 2 : 2));
}
}  // namespace

bool host_pinned(const void *p) {
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, const_cast<void *>(p), 0) == hipSuccess && dp) return true;
    (void)hipGetLastError();
    return false;
}

int copy_files_sync(int dev, hipStream_t stream, const Src *src, uint8_t *const *dst, uint32_t n) {
    std::vector<hipEvent_t> ev(1, nullptr);
    if (hipSetDevice(dev) != hipSuccess || hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess)
        return GCK_EDEVICE;
    int rc;
    {
        Copier cp;
        rc = cp.start(dev, stream, &ev);
        for (uint32_t f = 0; f < n && !rc; ++f) {
            if (!src[f].len) continue;
            if (src[f].data && host_pinned(src[f].data))
                rc = cp.direct(src[f].data, src[f].len, dst[f]);
            else
                cp.add(0, src[f], 0, src[f].len, dst[f]);
        }
        cp.seal(0);
        if (!rc) rc = cp.wait_recorded(0);
        const int r2 = cp.finish();
        if (!rc) rc = r2;
    }
    if (hipStreamSynchronize(stream) != hipSuccess && !rc) rc = GCK_EDEVICE;
    (void)hipEventDestroy(ev[0]);
    return rc;
}

std::vector<Src> mem_srcs(const gck_file *files, uint32_t nfiles) {
    std::vector<Src> v(nfiles);
    for (uint32_t f = 0; f < nfiles; ++f) v[f] = Src{files[f].data, nullptr, files[f].len, files[f].reset_after != 0, 0, 0};
    return v;
}

int open_srcs(const gck_path *files, uint32_t nfiles, std::vector<Src> &v) {
    v.assign(nfiles, Src{nullptr, nullptr, 0, false, 0, 0});
    for (uint32_t f = 0; f < nfiles; ++f) {
        struct stat st;
        if (!files[f].path || stat(files[f].path, &st) != 0 || !S_ISREG(st.st_mode)) {
            if (files[f].path) set_error("stat of a data file failed (missing, or not a regular file)", hipSuccess,
                                         __FILE__, __LINE__);
            v.clear();
            return GCK_EIO;
        }
        v[f].path = files[f].path;
        v[f].len = (uint64_t)st.st_size;
        v[f].reset_after = files[f].reset_after != 0;
        v[f].dev = (uint64_t)st.st_dev;
        v[f].ino = (uint64_t)st.st_ino;
    }
    return GCK_OK;
}

void close_srcs(std::vector<Src> &v) { v.clear(); }

uint32_t stage_buffers_wanted() { return 2 * copy_threads(); }

int stage_prealloc(int dev, uint32_t n) {
    std::vector<void *> b;
    if (hipSetDevice(dev) != hipSuccess) return GCK_EDEVICE;
    const int rc = stage_take(dev, n, b);
    std::lock_guard<std::mutex> lk(g_stage.mu);
    for (void *q : b) g_stage.idle.emplace_back(dev, q);
    return rc;
}

// Host arrays handed to callers in gck_result (recs, keys): page-locked
// (hipHostMalloc: D2H targets) or plain (malloc: assembled by the host from
// page-locked pieces -- pinning a 0.4 GB array at the end of an Open took
// 0.4-0.5 s); gck_result_free frees either.
namespace {
std::mutex g_res_mu;
std::unordered_set<void *> g_res_pinned;
}  // namespace

void *res_alloc(uint64_t bytes, bool pinned) {
    if (!bytes) bytes = 1;
    if (!pinned) {
        // large arrays the device copies into: huge pages where the kernel
        // offers them on request (THP "madvise"), so the first touch of a
        // GiB-sized result costs 512x fewer faults
        void *p = malloc(bytes);
        constexpr uintptr_t kHuge = 2ull << 20;
        if (p && bytes >= 4 * kHuge) {
            const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + kHuge - 1) & ~(kHuge - 1);
            const uintptr_t b = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(kHuge - 1);
            if (b > a) (void)madvise(reinterpret_cast<void *>(a), b - a, MADV_HUGEPAGE);
        }
        return p;
    }
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_res_mu);
    g_res_pinned.insert(p);
    return p;
}

void res_free(void *p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_res_mu);
        auto it = g_res_pinned.find(p);
        if (it != g_res_pinned.end()) {
            g_res_pinned.erase(it);
            (void)hipHostFree(p);
            return;
        }
    }
    free(p);
}

void par_gather(uint8_t *dst, const std::vector<std::pair<const void *, uint64_t>> &segs) {
    uint64_t total = 0;
    for (auto &s : segs) total += s.second;
    const uint32_t T = total >= (64ull << 20) ? copy_threads() : 1;
    auto part = [&](uint64_t lo, uint64_t hi) {  // destination bytes [lo, hi)
        uint64_t at = 0;
        for (auto &s : segs) {
            const uint64_t a = std::max(lo, at), b = std::min(hi, at + s.second);
            if (a < b) memcpy(dst + a, static_cast<const uint8_t *>(s.first) + (a - at), b - a);
            at += s.second;
            if (at >= hi) break;
        }
    };
    if (T == 1) {
        part(0, total);
        return;
    }
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; ++t) th.emplace_back(part, total * t / T, total * (t + 1) / T);
    for (auto &x : th) x.join();
}

void stage_release() {
    std::lock_guard<std::mutex> lk(g_stage.mu);
    for (auto &e : g_stage.idle) stage_free(e.second);
    g_stage.idle.clear();
}

struct Copier::Impl {
    struct Job {
        const uint8_t *src;  // caller memory, or nullptr: pread of path at off
        const char *path;
        uint64_t dev, ino;  // the file stat saw at path
        uint64_t off, len;
        uint8_t *dst;
        uint32_t group;
    };
    hipStream_t stream;
    std::vector<hipEvent_t> *group_ev;
    std::mutex mu;
    std::condition_variable cv_job, cv_group;
    std::deque<Job> jobs;
    std::vector<uint64_t> pending;   // per group: chunks not yet queued on the stream
    std::vector<uint8_t> recorded;   // per group: its event recorded after its last chunk
    std::vector<uint8_t> sealed;     // per group: every chunk submitted
    std::vector<void *> bufs;
    std::vector<hipEvent_t> buf_ev;  // per buffer: the last DMA out of it
    std::vector<uint8_t> buf_busy;
    std::vector<std::thread> workers;
    bool stop = false;
    int err = GCK_OK;

    // group g's event on the stream once its last chunk is queued (mu held)
    void maybe_record(uint32_t g) {
        if (!sealed[g] || pending[g] || recorded[g]) return;
        if (hipEventRecord((*group_ev)[g], stream) != hipSuccess && !err) err = GCK_EDEVICE;
        recorded[g] = 1;
        cv_group.notify_all();
    }

    void work() {
        for (;;) {
            Job j;
            size_t b = 0;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_job.wait(lk, [&] { return stop || !jobs.empty(); });
                if (jobs.empty()) return;
                j = jobs.front();
                jobs.pop_front();
                // a free staging buffer (one whose last DMA has finished)
                for (;;) {
                    bool found = false;
                    for (b = 0; b < bufs.size(); ++b)
                        if (!buf_busy[b]) {
                            found = true;
                            break;
                        }
                    if (found) break;
                    cv_job.wait(lk);
                }
                buf_busy[b] = 1;
            }
            (void)hipEventSynchronize(buf_ev[b]);  // the buffer's previous transfer
            uint8_t *stage = static_cast<uint8_t *>(bufs[b]);
            bool ok = true, replaced = false;
            if (j.src) {
                memcpy(stage, j.src + j.off, j.len);
            } else {
                // the file is opened per chunk: at most one descriptor per
                // copy thread is ever open.  Every chunk must come from the
                // file open_srcs stat'ed (a rename over the path or an unlink
                // and re-create in between would mix two files' bytes into
                // one image): otherwise GCK_EIO, like an unreadable file
                const int fd = open(j.path, O_RDONLY | O_CLOEXEC);
                uint64_t got = 0;
                ok = fd >= 0;
                struct stat st;
                if (ok && (fstat(fd, &st) != 0 || (uint64_t)st.st_dev != j.dev || (uint64_t)st.st_ino != j.ino)) {
                    ok = false;
                    replaced = true;
                }
                while (ok && got < j.len) {
                    const ssize_t r = pread(fd, stage + got, j.len - got, (off_t)(j.off + got));
                    if (r <= 0) {
                        ok = false;
                        break;
                    }
                    got += (uint64_t)r;
                }
                if (fd >= 0) close(fd);
            }
            std::lock_guard<std::mutex> lk(mu);
            if (!ok && !err) {  // the file shrank, could not be read, or was replaced
                err = GCK_EIO;
                set_error(replaced ? "a data file was replaced while it was read (another inode at its path)"
                                   : "pread of a data file failed (unreadable, or shorter than its stat size)",
                          hipSuccess, __FILE__, __LINE__);
            }
            if (ok && (hipMemcpyAsync(j.dst, stage, j.len, hipMemcpyHostToDevice, stream) != hipSuccess ||
                       hipEventRecord(buf_ev[b], stream) != hipSuccess) &&
                !err)
                err = GCK_EDEVICE;
            buf_busy[b] = 0;
            --pending[j.group];
            maybe_record(j.group);
            cv_job.notify_all();
        }
    }
};

Copier::Copier() : p(new Impl) {}
Copier::~Copier() {
    finish();
    for (auto e : p->buf_ev)
        if (e) (void)hipEventDestroy(e);
    delete p;
}

int Copier::start(int dev, hipStream_t stream, std::vector<hipEvent_t> *group_ev) {
    p->stream = stream;
    p->group_ev = group_ev;
    const size_t G = group_ev->size();
    p->pending.assign(G, 0);
    p->recorded.assign(G, 0);
    p->sealed.assign(G, 0);
    const uint32_t T = copy_threads();
    const size_t nb = stage_buffers_wanted();
    dev_ = dev;
    if (stage_take(dev, nb, p->bufs)) return GCK_ENOMEM;
    p->buf_ev.assign(nb, nullptr);
    p->buf_busy.assign(nb, 0);
    for (auto &e : p->buf_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return GCK_EDEVICE;
    for (uint32_t t = 0; t < T; ++t) p->workers.emplace_back([this] {
        (void)hipSetDevice(dev_);
        p->work();
    });
    return GCK_OK;
}

void Copier::add(uint32_t group, const Src &src, uint64_t off, uint64_t len, uint8_t *dst) {
    std::lock_guard<std::mutex> lk(p->mu);
    const uint64_t C = stage_chunk();
    for (uint64_t o = 0; o < len; o += C) {
        const uint64_t n = std::min(C, len - o);
        p->jobs.push_back(Impl::Job{src.data, src.path, src.dev, src.ino, off + o, n, dst + o, group});
        ++p->pending[group];
    }
    p->cv_job.notify_all();
}

int Copier::direct(const uint8_t *src, uint64_t len, uint8_t *dst) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (hipMemcpyAsync(dst, src, len, hipMemcpyHostToDevice, p->stream) != hipSuccess) return GCK_EDEVICE;
    return GCK_OK;
}

void Copier::seal(uint32_t group) {
    std::lock_guard<std::mutex> lk(p->mu);
    p->sealed[group] = 1;
    p->maybe_record(group);
}

int Copier::wait_recorded(uint32_t group) {
    std::unique_lock<std::mutex> lk(p->mu);
    p->cv_group.wait(lk, [&] { return p->recorded[group] || p->err; });
    return p->err;
}

int Copier::finish() {
    {
        std::lock_guard<std::mutex> lk(p->mu);
        p->stop = true;
        p->jobs.clear();  // (an error path: nothing waits for them any more)
        p->cv_job.notify_all();
    }
    for (auto &t : p->workers)
        if (t.joinable()) t.join();
    p->workers.clear();
    // the buffers go back once their last transfers are done
    for (auto e : p->buf_ev)
        if (e) (void)hipEventSynchronize(e);
    stage_give(dev_, p->bufs);
    return p->err;
}

}  // namespace gck

// replay.hip — MI355X (gfx950) cold-start replay of GoCask data files.
//
// Replaces (*DB).init / walkFile / readEntry (core/db.go:110-178) and the keydir
// offset arithmetic (core/keydir.go:22-53), and applies the lazy CRC rule of
// (*DB).get (core/db.go:311) to every record.  Pipeline:
//
//   k_spec_entry   one wavefront per 256 KiB chunk: first plausible record start
//   k_walk         one lane per chunk: speculative header chain, records staged
//   k_validate     chunk k's entry must equal chunk k-1's exit; k_fixup re-walks
//   k_scan_chunks  record slot per chunk (exclusive scan), per-file summary
//   (host)         EOF classification, lastOffset carries (core/db.go:117)
//   k_compact      record table (arena offset + header), walk order
//   k_row_tail     first record touching each 4 KiB row (with k_compact)
//   k_crc_rows     HBM-bound: every byte once, CRC partials of every value
//   k_finalize     CRC verdict, ValuePos (u32 wrap), gck_rec tuples
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "gck_internal.h"
#include "kd_common.h"
#include "gck_crc_lds.h"
#include "gck_crc_wave.h"

namespace gck {

static thread_local std::string g_err;
void set_error(const char *what, hipError_t e, const char *file, int line) {
    char buf[512];
    snprintf(buf, sizeof buf, "%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
    g_err = buf;
}
const char *last_error() { return g_err.c_str(); }

enum : uint32_t { T_NONE = 0, T_SILENT = 1, T_ERR = 2 };
// Counter slots (d_counters, u32): 1 fixups, 2 chunks whose stage overflowed
// (re-walked by k_compact), 3 CRC rejects, 6 record-table capacity overflow,
// 8.. validation rounds, 12-13 finalize's arrivals and rejects (one u64: the
// device path's publish), 5 the settle rounds' grid barrier, 14 the diag
// kernels' sink, 15 host validation loop.
enum : int {
    CNT_FIXUP = 1, CNT_STAGE = 2, CNT_REJECT = 3, CNT_BAR = 5, CNT_CAP = 6, CNT_VAL = 8, CNT_FINTICKET = 12,
    CNT_HOSTVAL = 15
};
constexpr int kRounds = 2;             // device validation/fixup rounds
constexpr int kHops = 4;          // extra headers a speculative start must chain through
#ifndef GCK_CRC_WAVES
#define GCK_CRC_WAVES 16
#endif
constexpr int kWaves = GCK_CRC_WAVES;  // wavefronts per k_crc_rows workgroup (one workgroup per CU: its LDS)
constexpr uint32_t kNibBase = 32768;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

// Diagnostic build only (make EXTRA=-DGCK_CLOCK_STAMPS OUT=../var/...): every
// wavefront of k_crc_rows, k_clk_stream, k_spec_entry, k_walk, k_compact and
// k_finalize stamps the shader clock and the
// 100 MHz real-time counter when its loop starts and when it leaves, into
// buffers of their own that nothing else reads; the in-kernel clock is
// d(shader clock) / d(real time) x 100 MHz (MI355X_MICROARCH.md, DVFS item 6).
// gck_xp_clock() reads them back.  The product build has no stamp.
#ifdef GCK_CLOCK_STAMPS
constexpr uint32_t kClkWaves = 65536;  // k_spec_entry and k_compact run 65,536 wavefronts on C3
constexpr int kClkKinds = 6;  // 0 k_crc_rows, 1 k_clk_stream, 2 k_spec_entry, 3 k_walk, 4 k_compact, 5 k_finalize
__device__ uint64_t g_clk[kClkKinds][4 * kClkWaves];
__device__ uint32_t g_clk_xcc[kClkKinds][kClkWaves];
__device__ uint64_t g_fin_split[2 * kClkWaves];  // k_finalize: (wait, compute) cycles per wavefront
__device__ __forceinline__ void clk_put(int which, uint32_t wi, uint64_t t0, uint64_t r0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0 && wi < kClkWaves) {
        g_clk_xcc[which][wi] = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;  // HW_REG_XCC_ID[3:0]
        u32x4 a, b;
        a.x = (uint32_t)t0, a.y = (uint32_t)(t0 >> 32), a.z = (uint32_t)r0, a.w = (uint32_t)(r0 >> 32);
        b.x = (uint32_t)t1, b.y = (uint32_t)(t1 >> 32), b.z = (uint32_t)r1, b.w = (uint32_t)(r1 >> 32);
        u32x4 *d = reinterpret_cast<u32x4 *>(&g_clk[which][4 * wi]);
        d[0] = a;
        d[1] = b;
    }
}
#define GCK_CLK_BEGIN() const uint64_t clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime()
#define GCK_CLK_END(which, wi) clk_put(which, wi, clk_t0, clk_r0)
#else
#define GCK_CLK_BEGIN() ((void)0)
#define GCK_CLK_END(which, wi) ((void)0)
#endif


// ---------------------------------------------------------------- helpers ---

// Raw buffer resource over [p, p + bytes) (gfx9 dword3: untyped, bounds-checked).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ uint32_t ab(uint32_t hi, uint32_t lo, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

struct Hdr {
    uint32_t crc, ts, ks, vs;
};

// 16-byte little-endian header at any byte offset (core/header.go:58-62).  The
// arena is 4 KiB aligned and padded, so the 5-dword over-read stays in bounds.
__device__ __forceinline__ Hdr ld_hdr(const uint8_t *__restrict__ arena, uint64_t o) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(arena + (o & ~3ull));
    const uint32_t sh = (uint32_t)o & 3u;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    Hdr h;
    h.crc = ab(w1, w0, sh);
    h.ts = ab(w2, w1, sh);
    h.ks = ab(w3, w2, sh);
    h.vs = ab(w4, w3, sh);
    return h;
}

// Follow the header chain from q for kHops+1 headers: key length in
// [1, max_key] and every record inside the file.  A chain may only end exactly
// at the file end.  (A record straddling the file end is rejected: that only
// costs a fixup for the one chunk where it is real.)
__device__ bool chain_ok(const uint8_t *__restrict__ arena, uint64_t base, uint64_t len, uint64_t q,
                         uint32_t max_key) {
    for (int h = 0; h <= kHops; ++h) {
        if (q == len) return h > 0;
        if (q + 16 > len) return false;
        const Hdr hd = ld_hdr(arena, base + q);
        const uint32_t klen = hd.ks ? hd.ks : hd.vs;
        if (klen == 0 || klen > max_key) return false;
        const uint64_t end = q + 16 + (uint64_t)hd.ks + hd.vs;
        if (end > len) return false;
        q = end;
    }
    return true;
}

// The reference's readEntry loop (core/db.go:131-178) over one chunk: decode
// headers from p while p < ce.  EOF classes follow Go's io.ReadFull /
// bufio.Reader.Discard semantics.  emit(i, p, hdr) per record.
template <class Emit>
__device__ void walk_chain(const uint8_t *__restrict__ arena, uint64_t base, uint64_t len, uint64_t ce,
                           uint64_t p, Emit emit, uint32_t &count, uint64_t &exit, uint32_t &term,
                           uint64_t &tpos) {
    auto ld = [&](uint64_t o) { return ld_hdr(arena, o); };
    uint32_t n = 0;
    term = T_NONE;
    tpos = 0;
    // Software-pipelined: the next header's loads are issued before this
    // record's stores, so a hop waits for one load latency, never for the
    // previous hop's store acknowledgements (vmcnt counts both, in order).
    // base / len are consumed here, before the loop, so no load issued
    // outside the loop is still pending inside it.
    const uint64_t a0 = base + (p < len ? p : 0);
    Hdr h = ld(a0);
    emit.prime();  // the loop is entered with the back edge's queue shape
    while (p < ce) {
        const uint64_t rem = len - p;
        if (rem < 16) { term = T_ERR; tpos = p; break; }            // ErrUnexpectedEOF
        const uint32_t klen = h.ks ? h.ks : h.vs;                    // db.go:151-155
        const uint64_t rem2 = rem - 16;
        if (klen > 0 && rem2 == 0) { term = T_SILENT; tpos = p; break; }  // ReadFull io.EOF
        if (rem2 < klen) { term = T_ERR; tpos = p; break; }          // partial key
        uint64_t next;
        if (h.ks == 0) {
            next = p + 16 + klen;                                    // tombstone
        } else {
            if (rem2 - klen < h.vs) { term = T_SILENT; tpos = p; break; }  // Discard io.EOF
            next = p + 16 + (uint64_t)h.ks + h.vs;
        }
        // the next header (the arena is padded: a read at the file end or
        // just past the chunk stays in bounds and is never used)
        const Hdr hn = ld(base + (next < len ? next : 0));
        emit(n, p, h);
        ++n;
        p = next;
        h = hn;
    }
    count = n;
    exit = p;
}

// ------------------------------------------------------------------ kernels ---
#ifndef GCK_SPEC_DOT
#define GCK_SPEC_DOT 1
#endif
// Bit 7 of each byte of the result is set iff that byte of w is zero (exact).
__device__ __forceinline__ uint32_t zero_bytes(uint32_t w) {
    return ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w | 0x7F7F7F7Fu);
}

// One wavefront per chunk finds the first byte position p in [chunk start,
// chunk start + window) whose header and the next kHops headers are plausible
// (chunk 0 of a file starts at 0); none (kNone) when no position in the window
// qualifies: the walk of the chunk before then covers this chunk too.  Chunk
// starts inside long values (most of the corpus bytes sit in values > 4 KiB)
// would otherwise stream the rest of the value; a bounded window keeps the
// search cost per chunk fixed, so chunks can be small (short walk chains)
// where records are dense, and merge where they are sparse (few hops).  Each
// pass covers 4 KiB of positions, 64 per lane.  Prefilter: a header
// at p with KeySize <= 65535 (tombstones: KeySize 0) has bytes p+10 and p+11
// zero, so the lane flags positions whose bytes 10, 11 are a zero pair (about
// 2 VALU per position; in value bytes a zero pair is rare) and only flagged
// positions get the full chain test.  A hit at p is replaced by p+k (k <= 3,
// the largest that chains): a true header has plausible "shadows" 1..3 bytes
// earlier (Timestamp's top bytes + KeySize shifted).  Keys longer than 65535
// bytes are never speculated here; validation finds their chunks and re-walks.
__device__ void spec_chunk(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ fbase,
                           const uint64_t *__restrict__ flen, const uint32_t *__restrict__ ch_file,
                           const uint64_t *__restrict__ ch_start, const uint64_t *__restrict__ ch_end,
                           uint64_t *__restrict__ ch_entry, uint32_t c, uint32_t max_key, uint64_t window) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t f = ch_file[c];
    const uint64_t cs = ch_start[c], ce = ch_end[c], base = fbase[f], len = flen[f];
    const uint32_t mk = min(max_key, 65535u);
    uint64_t found = kNone;
    if (cs == 0) {
        found = 0;
    } else {
        // The scan loop only computes candidate masks (no dependent loads in
        // it, so the next window's loads stay in flight: windows A/B rotate,
        // unrolled so none is copied); a window with candidates leaves the
        // loop for the chain tests and the scan resumes after it if none holds.
        // Lane L scans positions [64 L, 64 L + 64) of a 4 KiB window and
        // needs bytes [64 L, 64 L + 80).  Loads as k_crc_rows': lane p + 16 b
        // reads 1024 k + 64 p + 16 b (k < 4: each instruction one contiguous
        // KiB, whole lines, non-temporal), the permlane transpose gives lane L
        // its 64 bytes, lane L + 1's first block (DPP) its last 16, and lane
        // 63 the window's next 16 bytes from a fifth load (one line, every
        // lane the same address).
        const uint32_t s_rel = 64 * (lane & 15) + 16 * (lane >> 4);
        auto load = [&](uint64_t b0, u32x4 (&v)[5]) {
            // (the arena is padded 3 windows past every file).  Buffer loads:
            // the compiler keeps them where they are issued (ahead of their use).
            const __amdgpu_buffer_rsrc_t rw = make_rsrc(arena + base + b0, 4096 + 80);
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rw, s_rel + 1024 * k, 0, 2);
            v[4] = __builtin_amdgcn_raw_buffer_load_b128(rw, 4096, 0, 0);
        };
        auto cands = [&](const u32x4 (&v)[5]) -> uint64_t {  // bit t: bytes p0+t+10, p0+t+11 both zero
            uint32_t w[20];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                w[4 * k] = v[k].x;
                w[4 * k + 1] = v[k].y;
                w[4 * k + 2] = v[k].z;
                w[4 * k + 3] = v[k].w;
            }
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const auto r = __builtin_amdgcn_permlane32_swap(w[4 * k + c4], w[4 * (k + 2) + c4], false, false);
                    w[4 * k + c4] = r[0];
                    w[4 * (k + 2) + c4] = r[1];
                }
            }
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
#pragma unroll
                for (int k = 0; k < 4; k += 2) {
                    const auto r = __builtin_amdgcn_permlane16_swap(w[4 * k + c4], w[4 * (k + 1) + c4], false, false);
                    w[4 * k + c4] = r[0];
                    w[4 * (k + 1) + c4] = r[1];
                }
            }
            // bytes 64 L + 64 .. 79: lane L + 1's first block (wave_shl:1), lane 63 the fifth load
            w[16] = (uint32_t)__builtin_amdgcn_update_dpp((int)v[4].x, (int)w[0], 0x130, 0xF, 0xF, false);
            w[17] = (uint32_t)__builtin_amdgcn_update_dpp((int)v[4].y, (int)w[1], 0x130, 0xF, 0xF, false);
            w[18] = (uint32_t)__builtin_amdgcn_update_dpp((int)v[4].z, (int)w[2], 0x130, 0xF, 0xF, false);
            w[19] = (uint32_t)__builtin_amdgcn_update_dpp((int)v[4].w, (int)w[3], 0x130, 0xF, 0xF, false);
#if GCK_SPEC_DOT
            // nz(k): bit 7 of byte j set iff bytes 4k+j, 4k+j+1 are not both
            // zero (x = the word OR'ed with itself one byte on; a zero byte of
            // x = a zero pair).  Two words' flags become one byte with two
            // v_dot4_u32_u8 (flag 0x80 times 1, 2, 4, ..., 128, summed): byte j of
            // the 72-bit m = words 2 + 2j, 3 + 2j; position t = bit u of m - 2.
            // The candidates are the complement.  About 7 VALU per word where
            // the per-bit nibble gather took 15 (k_spec_entry is VALU-bound
            // about half its cycles, profiles/r5end2 PMC)
            auto nz = [&](int k) {
                const uint32_t x = w[k] | __builtin_amdgcn_alignbyte(w[k + 1], w[k], 1);
                return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
            };
            uint32_t mb[9];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                mb[j] = __builtin_amdgcn_udot4(nz(2 + 2 * j), 0x08040201u,
                                               __builtin_amdgcn_udot4(nz(3 + 2 * j), 0x80402010u, 0u, false), false) >> 7;
            mb[8] = __builtin_amdgcn_udot4(nz(18), 0x08040201u, 0u, false) >> 7;
            const uint32_t lo = mb[0] | (mb[1] << 8) | (mb[2] << 16) | (mb[3] << 24);
            const uint32_t hi = mb[4] | (mb[5] << 8) | (mb[6] << 16) | (mb[7] << 24);
            const uint32_t r0 = __builtin_amdgcn_alignbit(hi, lo, 2), r1 = __builtin_amdgcn_alignbit(mb[8], hi, 2);
            return ~(((uint64_t)r1 << 32) | r0);
#else
            uint32_t zf[20];
#pragma unroll
            for (int k = 2; k < 20; ++k) zf[k] = zero_bytes(w[k]);
            uint64_t cm = 0;
#pragma unroll
            for (int k = 2; k <= 18; ++k) {
                const uint32_t pr = zf[k] & ((zf[k] >> 8) | (zf[k + 1] << 24));
                const uint32_t nib = ((pr >> 7) & 1u) | ((pr >> 14) & 2u) | ((pr >> 21) & 4u) | ((pr >> 28) & 8u);
                const int t0 = 4 * k - 10;
                cm |= t0 >= 0 ? (uint64_t)nib << t0 : (uint64_t)(nib >> -t0);
            }
            return cm;
#endif
        };
        // positions searched: [cs, lim).  The next window is loaded one ahead,
        // unconditionally (the arena is padded past every file; a branch
        // around a load would cost the prefetch its place).  Two ahead read a
        // sixth more (a chunk's entry is 4.3 windows in on C3, the prefetch
        // past it is wasted) and measured 2 % slower: 0.289-0.291 against
        // 0.284 ms; the first window alone before any prefetch, 0.302-0.310.
        const uint64_t lim = ce - cs > window ? cs + window : ce;
        uint64_t from = cs;
        while (found == kNone && from < lim) {
            uint64_t wb = kNone, cm = 0;
            u32x4 A[5], B[5];
            load(from, A);
            for (uint64_t b0 = from;; b0 += 2 * 4096) {
                load(b0 + 4096, B);
                cm = cands(A);
                if (__ballot(cm != 0)) { wb = b0; break; }
                if (b0 + 4096 >= lim) break;
                load(b0 + 2 * 4096, A);
                cm = cands(B);
                if (__ballot(cm != 0)) { wb = b0 + 4096; break; }
                if (b0 + 2 * 4096 >= lim) break;
            }
            if (wb == kNone) break;
            // Candidates in scan order are lane l's bits, then lane l + 1's.
            // Every lane tests its own candidates in order, all lanes at once
            // (a chain test is 5 dependent header loads: in turn, one lane's
            // candidates after another's made the search latency-bound); the
            // answer is the first passing candidate of the lowest lane with
            // one, so lanes above the lowest that has passed stop.
            uint64_t lm = cm, mine = kNone;
            for (uint64_t pend = __ballot(lm != 0); pend;) {
                const uint64_t passed = __ballot(mine != kNone);
                const uint64_t go = passed ? pend & ((passed & (0 - passed)) - 1) : pend;
                if (!go) break;
                if ((go >> lane) & 1) {
                    const int t = __ffsll((long long)lm) - 1;
                    const uint64_t q = wb + 64ull * lane + t;
                    if (q < ce && chain_ok(arena, base, len, q, mk)) mine = q;
                    lm &= lm - 1;
                }
                pend = __ballot(lm != 0 && mine == kNone);
            }
            const uint64_t passed = __ballot(mine != kNone);
            if (passed) {
                const int L = __builtin_ctzll(passed);
                found = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mine >> 32), L) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mine, L);
            }
            from = wb + 4096;
        }
        // shadows: next to a true header at p, positions p-2, p-1 (KeySize =
        // the timestamp's high bytes plus KeySize << 8) and p+3 (KeySize =
        // ValueSize << 8) often decode as plausible headers too, and one long
        // first hop can land such a shadow on the true chain, which then
        // chains.  A shadow's fields are the true ones shifted by whole
        // bytes, so its first hop is >= 256 times the true record's: of the
        // chaining positions within 3 bytes of the first one, the one with
        // the shortest first record wins (ties: the earliest).  (Preferring
        // the latest mis-speculated ~5 chunks of C3's 65 K, the earliest ~15.)
        if (found != kNone) {
            // lanes 0..3 take found + lane at once: its first hop, kept if it
            // chains (found itself does); the shortest wins, ties the earliest
            uint64_t hop = ~0ull;
            if (lane <= 3 && found + lane < ce) {
                const Hdr hk = ld_hdr(arena, base + found + lane);
                const uint64_t h = 16ull + hk.ks + hk.vs;
                if (lane == 0 || chain_ok(arena, base, len, found + lane, mk)) hop = h;
            }
            uint64_t best = ~0ull, pick = found;
#pragma unroll
            for (int k = 0; k <= 3; ++k) {
                const uint64_t hk = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(hop >> 32), k) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hop, k);
                if (hk < best) {
                    best = hk;
                    pick = found + k;
                }
            }
            found = pick;
        }
    }
    if (lane == 0) ch_entry[c] = found;
}

// The device path's per-run zeroing (counters / results, record base and
// ranges, row_first[0], the CRC block queue), done by k_spec_entry's first
// wavefront: nothing reads them before the walk, and a separate k_run_init
// launch cost ~2.5 us plus a dispatch per step.  cnt == nullptr: not asked.
struct RunInit {
    uint32_t *cnt;
    uint64_t *gb;
    uint32_t *blk_first;
    uint32_t *queue;
};
__device__ __forceinline__ void run_init(const RunInit &ri, uint32_t t) {
    if (t < 32) ri.cnt[t] = 0;
    if (t < kGbWords) ri.gb[t] = 0;
    if (t == kQueueCrc) ri.queue[t] = 0;
    if (t == 0) ri.blk_first[0] = 0;
}

__global__ __launch_bounds__(256) void k_spec_entry(const uint8_t *__restrict__ arena,
                                                    const uint64_t *__restrict__ fbase,
                                                    const uint64_t *__restrict__ flen,
                                                    const uint32_t *__restrict__ ch_file,
                                                    const uint64_t *__restrict__ ch_start,
                                                    const uint64_t *__restrict__ ch_end,
                                                    uint64_t *__restrict__ ch_entry, uint32_t n_chunks,
                                                    uint32_t max_key, uint64_t window, RunInit ri) {
    if (ri.cnt && blockIdx.x == 0 && threadIdx.x < 64) run_init(ri, threadIdx.x);
    const uint32_t c = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));  // wave-uniform
    if (c >= n_chunks) return;
    GCK_CLK_BEGIN();
    spec_chunk(arena, fbase, flen, ch_file, ch_start, ch_end, ch_entry, c, max_key, window);
    GCK_CLK_END(2, c);
}

// The stage: per chunk, cap record slots + 1 scratch slot (records past cap
// land there; k_compact re-walks such chunks), interleaved over groups of
// kStageIl consecutive chunks: slot i of chunk c is element
// ((c / kStageIl) * (cap + 1) + i) * kStageIl + c % kStageIl.  The lanes of a
// k_walk wavefront walk consecutive chunks hop by hop, so a hop's stage store
// writes 64 / kStageIl runs of kStageIl consecutive elements (whole lines)
// instead of 64 scattered partial lines (measured: those cost half of the
// walk), and k_compact still reads a chunk's slots at a short stride.
constexpr uint32_t kStageIl = 8;
#ifndef GCK_PRE_BATCHES
#define GCK_PRE_BATCHES 3
#endif
constexpr uint32_t kPreBatches = GCK_PRE_BATCHES;  // stage batches of 64 k_compact loads up front (C3: 154 records per chunk on average)
__host__ __device__ __forceinline__ uint64_t stage_slot(uint32_t c, uint32_t i, uint32_t cap) {
    return ((uint64_t)(c / kStageIl) * (cap + 1) + (i < cap ? i : cap)) * kStageIl + (c % kStageIl);
}
// Every hop stores, so the number of stores per hop is fixed and the next
// header's load wait counts them.  A slot holds (KeySize, ValueSize): the
// record offsets follow from the chunk's entry and the entry sizes (a scan in
// k_compact), CRC and Timestamp from the header bytes (k_finalize reads them).
struct ScratchEmit {
    uint2 *kv;  // the chunk's slot 0 (stride kStageIl elements)
    uint32_t cap;
    __device__ void operator()(uint32_t i, uint64_t, const Hdr &h) const {
        kv[(uint64_t)(i < cap ? i : cap) * kStageIl] = make_uint2(h.ks, h.vs);
    }
    // the store of one hop, to the scratch slot
    __device__ void prime() const { kv[(uint64_t)cap * kStageIl] = make_uint2(0, 0); }
};

// Where the walk of chunk c stops: the start of the next chunk of its file
// that has an entry (its records are that chunk's), else the file end.  A
// chunk without an entry is covered by the walk of the nearest earlier chunk
// that has one.  Chunk starts are (index within the file) << chunk_shift.
// *nxt = that chunk (the file's chunk end fe if none), *nentry = its entry.
__device__ uint64_t walk_bound(const uint64_t *ch_entry, const uint32_t *__restrict__ f_first_chunk,
                               const uint32_t *__restrict__ f_nchunks, const uint64_t *__restrict__ flen, uint32_t c,
                               uint32_t f, uint32_t chunk_shift, uint32_t *nxt = nullptr, uint64_t *nentry = nullptr) {
    const uint32_t fc = f_first_chunk[f], fe = fc + f_nchunks[f];
    for (uint32_t d = c + 1; d < fe; d += 4) {
        uint64_t e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = d + k < fe ? ch_entry[d + k] : kNone;  // 4 loads in flight
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (e[k] != kNone) {
                if (nxt) *nxt = d + k;
                if (nentry) *nentry = e[k];
                return (uint64_t)(d + k - fc) << chunk_shift;
            }
    }
    if (nxt) *nxt = fe;
    return flen[f];
}

__device__ void walk_into_chunk(const uint8_t *__restrict__ arena, const uint64_t *fbase,
                                const uint64_t *flen, uint32_t c, uint32_t f, uint64_t ce, uint64_t entry,
                                uint32_t cap, uint2 *s_kv, uint32_t *ch_count,
                                uint64_t *ch_exit, uint32_t *ch_term, uint64_t *ch_tpos, uint64_t *ch_wend,
                                uint64_t *ch_aentry) {
    uint32_t count = 0, term = T_NONE;
    uint64_t exit = kNone, tpos = 0, aentry = 0;
    if (entry != kNone) {
        ScratchEmit em{s_kv + stage_slot(c, 0, cap), cap};
        const uint64_t base = fbase[f];
        aentry = base + entry;
        walk_chain(arena, base, flen[f], ce, entry, em, count, exit, term, tpos);
    }
    ch_aentry[c] = aentry;
    ch_count[c] = count;
    ch_exit[c] = exit;
    ch_term[c] = term;
    ch_tpos[c] = tpos;
    ch_wend[c] = ce;
}

// One lane per chunk of [c_begin, c_end): latency-bound header chain from the
// speculative entry to the walk bound (walk_bound).  With val (the device
// path) the walk also does validation round 0 (k_validate's verdicts, counted
// in *val): a lane with an entry knows the next chunk of its file that has
// one, c' (walk_bound found it), and its own exit, so it decides c' (bad iff
// its walk ended at an EOF or exit != entry of c'); the chunks between them
// have no entry and are covered (the walk went past their ends, or ended at
// an EOF), so never bad, as a file's first chunk.  Each chunk's flag is
// written once: by its own lane (no entry, or a file's first chunk) or by
// the lane of its predecessor with an entry.  One launch fewer per step.
__global__ __launch_bounds__(256) void k_walk(const uint8_t *__restrict__ arena,
                                              const uint64_t *__restrict__ fbase,
                                              const uint64_t *__restrict__ flen,
                                              const uint32_t *__restrict__ ch_file,
                                              const uint32_t *__restrict__ f_first_chunk,
                                              const uint32_t *__restrict__ f_nchunks,
                                              const uint64_t *__restrict__ ch_entry, uint32_t *ch_count,
                                              uint64_t *ch_exit, uint32_t *ch_term, uint64_t *ch_tpos,
                                              uint64_t *ch_wend, uint64_t *ch_aentry, uint2 *s_kv, uint32_t cap,
                                              uint32_t chunk_shift, uint32_t c_begin, uint32_t c_end,
                                              uint32_t *__restrict__ ch_bad, uint32_t *__restrict__ val) {
    GCK_CLK_BEGIN();
    const uint32_t c = c_begin + blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= c_end) return;
    const uint32_t f = ch_file[c];
    const uint64_t entry = ch_entry[c];
    uint32_t nxt = 0;
    uint64_t nentry = kNone;
    const uint64_t ce =
        entry != kNone ? walk_bound(ch_entry, f_first_chunk, f_nchunks, flen, c, f, chunk_shift, &nxt, &nentry) : 0;
    uint32_t count = 0, term = T_NONE;
    uint64_t exit = kNone, tpos = 0, aentry = 0;
    if (entry != kNone) {
        ScratchEmit em{s_kv + stage_slot(c, 0, cap), cap};
        const uint64_t base = fbase[f];
        aentry = base + entry;
        walk_chain(arena, base, flen[f], ce, entry, em, count, exit, term, tpos);
    }
    ch_aentry[c] = aentry;
    ch_count[c] = count;
    ch_exit[c] = exit;
    ch_term[c] = term;
    ch_tpos[c] = tpos;
    ch_wend[c] = ce;
    if (val) {
        const uint32_t fc = f_first_chunk[f], fe = fc + f_nchunks[f];
        if (entry == kNone || c == fc) ch_bad[c] = 0u;
        bool bad = false;
        if (entry != kNone && nxt < fe) {
            bad = term != T_NONE || exit != nentry;
            ch_bad[nxt] = bad ? 1u : 0u;
        }
        const uint64_t m = __ballot(bad);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(val, (uint32_t)__popcll(m));
    }
    GCK_CLK_END(3, (c - c_begin) >> 6);
}

// Consistency of chunk c against j, the nearest earlier chunk of its file with
// an entry (chunk 0 of a file always has one, entry 0): if c has an entry, j's
// walk must have ended exactly there (exit == entry, not at an EOF); if c has
// none, j's walk must have covered c (exit past c's end, or an EOF: then no
// later record exists).  If every chunk is consistent, every chunk is correct:
// induction over the chunk order from each file's chunk 0.  (Plain pointers:
// k_scan_chunks' settle rounds run this after fixups of the same launch.)
__device__ bool validate_chunk(uint32_t c, const uint32_t *ch_file, const uint64_t *ch_end, const uint64_t *ch_entry,
                               const uint64_t *ch_exit, const uint32_t *ch_term, const uint32_t *f_first_chunk,
                               uint32_t *ch_bad) {
    const uint32_t f = ch_file[c], fc = f_first_chunk[f];
    bool bad = false;
    if (c != fc) {
        uint32_t j = c - 1;
        while (j > fc && ch_entry[j] == kNone) --j;
        const bool ended = ch_entry[j] == kNone || ch_term[j] != T_NONE;
        const uint64_t x = ch_exit[j], e = ch_entry[c];
        bad = e != kNone ? (ended || x != e) : (!ended && x < ch_end[c]);
    }
    ch_bad[c] = bad ? 1u : 0u;
    return bad;
}
__global__ __launch_bounds__(256) void k_validate(const uint32_t *__restrict__ ch_file,
                                                  const uint64_t *__restrict__ ch_end,
                                                  const uint64_t *__restrict__ ch_entry,
                                                  const uint64_t *__restrict__ ch_exit,
                                                  const uint32_t *__restrict__ ch_term,
                                                  const uint32_t *__restrict__ f_first_chunk,
                                                  uint32_t *__restrict__ ch_bad, uint32_t *counter,
                                                  uint32_t c_begin, uint32_t c_end,
                                                  const uint32_t *__restrict__ prev_counter) {
    // a round after one that found every chunk consistent (so its fixup
    // changed nothing) finds the same: its counter stays at the run's zero
    if (prev_counter && *prev_counter == 0) return;
    const uint32_t c = c_begin + blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= c_end) return;
    const bool bad = validate_chunk(c, ch_file, ch_end, ch_entry, ch_exit, ch_term, f_first_chunk, ch_bad);
    const uint64_t m = __ballot(bad);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(counter, (uint32_t)__popcll(m));
}

// One lane per inconsistent chunk: its entry becomes the exit of the nearest
// earlier chunk with an entry (none if that walk ended at an EOF or went past
// this chunk), then it walks to its bound.  Chunks whose look-back crosses
// another inconsistent chunk wait for a later round (the next k_validate
// decides), so no lane reads state another lane is rewriting: the chunks a
// fixed chunk's walk_bound reads all look back to it and wait.
__device__ void fixup_chunk(uint32_t c, const uint8_t *__restrict__ arena, const uint64_t *fbase, const uint64_t *flen,
                            const uint32_t *ch_file, const uint64_t *ch_end, const uint32_t *f_first_chunk,
                            const uint32_t *f_nchunks, const uint32_t *ch_bad, uint64_t *ch_entry, uint32_t *ch_count,
                            uint64_t *ch_exit, uint32_t *ch_term, uint64_t *ch_tpos, uint64_t *ch_wend,
                            uint64_t *ch_aentry, uint2 *s_kv, uint32_t cap, uint32_t chunk_shift, uint32_t *counter) {
    const uint32_t f = ch_file[c], fc = f_first_chunk[f];
    uint32_t j = c - 1;
    while (j > fc && ch_entry[j] == kNone && !ch_bad[j]) --j;
    if (ch_bad[j] || ch_entry[j] == kNone) return;
    uint64_t e_new = kNone;
    if (ch_term[j] == T_NONE) {
        const uint64_t x = ch_exit[j];
        if (x < ch_end[c]) e_new = x;
    }
    ch_entry[c] = e_new;
    atomicAdd(counter, 1u);
    const uint64_t ce = e_new != kNone ? walk_bound(ch_entry, f_first_chunk, f_nchunks, flen, c, f, chunk_shift) : 0;
    walk_into_chunk(arena, fbase, flen, c, f, ce, e_new, cap, s_kv, ch_count, ch_exit, ch_term, ch_tpos,
                    ch_wend, ch_aentry);
}
__global__ __launch_bounds__(256) void k_fixup(const uint8_t *__restrict__ arena,
                                               const uint64_t *__restrict__ fbase,
                                               const uint64_t *__restrict__ flen,
                                               const uint32_t *__restrict__ ch_file,
                                               const uint64_t *__restrict__ ch_end,
                                               const uint32_t *__restrict__ f_first_chunk,
                                               const uint32_t *__restrict__ f_nchunks,
                                               const uint32_t *__restrict__ ch_bad, uint64_t *ch_entry,
                                               uint32_t *ch_count, uint64_t *ch_exit, uint32_t *ch_term,
                                               uint64_t *ch_tpos, uint64_t *ch_wend, uint64_t *ch_aentry, uint2 *s_kv,
                                               uint32_t cap, uint32_t chunk_shift, uint32_t c_begin, uint32_t c_end,
                                               uint32_t *counter, const uint32_t *__restrict__ bad_counter) {
    if (bad_counter && *bad_counter == 0) return;  // nothing to fix (the common case)
    const uint32_t c = c_begin + blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= c_end || !ch_bad[c]) return;
    fixup_chunk(c, arena, fbase, flen, ch_file, ch_end, f_first_chunk, f_nchunks, ch_bad, ch_entry, ch_count, ch_exit,
                ch_term, ch_tpos, ch_wend, ch_aentry, s_kv, cap, chunk_shift, counter);
}

// Exclusive scan of per-chunk record counts -> rec_base[0..n] (one wavefront
// per block of kScanBlock counts).
constexpr uint32_t kScanBlock = 4096;

// Inclusive prefix sum over the 64 lanes (DPP row shifts + row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// 64-bit inclusive prefix sum over the lanes (values < 2^48: two 24-bit halves)
__device__ __forceinline__ uint64_t wave_incl_sum64(uint64_t v) {
    const uint32_t lo = wave_incl_sum((uint32_t)(v & 0xFFFFFFu)), hi = wave_incl_sum((uint32_t)(v >> 24));
    return ((uint64_t)hi << 24) + lo;
}
// 64-bit value of lane 63 in every lane
__device__ __forceinline__ uint64_t lane63(uint64_t v) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}

// The host bookkeeping of a run (core/db.go:110-140) on the device, so a run
// needs no host round trip.  Per file the lastOffset carried in (reset after
// every file but the active one, core/db.go:117-119), the first startup error
// (it aborts filepath.Walk: later files contribute nothing, disk.go:134-141),
// the record range and the run's results.  One lane; res (u64): 0 status,
// 1 error file, 2 error offset, 3 files walked, 4 final lastOffset, 5 records
// (unclamped); grng = the record range [0, hi) clamped to cap, rng the same.
__device__ void account_run(uint32_t nf, const uint64_t *__restrict__ flen, const uint32_t *__restrict__ freset,
                            const uint32_t *fterm, const uint64_t *ftpos, const uint64_t *ffirst,
                            const uint64_t *fnrec, uint32_t *__restrict__ carry, uint64_t cap,
                            uint64_t *__restrict__ res, uint64_t *__restrict__ grng, uint64_t *__restrict__ rng,
                            bool unsettled) {
    uint32_t last = 0, walked = nf;
    uint64_t n_end = 0;
    for (uint32_t f = 0; f < nf; ++f) {
        carry[f] = last;
        const uint64_t valid = fterm[f] != T_NONE ? ftpos[f] : flen[f];
        n_end = ffirst[f] + fnrec[f];
        last += (uint32_t)valid;
        if (fterm[f] == T_ERR) {
            res[0] = GCK_EUNEXPECTED_EOF;
            res[1] = f;
            res[2] = ftpos[f];
            walked = f + 1;
            break;
        }
        if (freset[f]) last = 0;
    }
    res[3] = walked;
    res[4] = last;
    res[5] = n_end;
    grng[0] = 0;
    grng[1] = n_end < cap ? n_end : cap;
    // chunks left inconsistent by the settle rounds: the run is redone on the
    // host path; an empty range keeps finalize from reading the table
    if (unsettled) grng[1] = 0;
    rng[0] = 0;
    rng[1] = grng[1];
}

// account_run for up to 64 files, lane f holding file f's summary (its
// terminal condition and position, first record, records): the lastOffset
// carries are an exclusive prefix sum of the files' valid lengths (u32, as
// the reference's uint32 offsets wrap) restarted after every file that
// resets, and the first startup error cuts the walk, by wave scans instead of
// one lane's loop over the files (each iteration's loads waited behind the
// stores of the one before: ~10 us of the scan kernel's 14 on C3).
__device__ void account_run_wave(uint32_t nf, uint32_t lane, uint32_t term, uint64_t tpos, uint64_t r0, uint64_t nrec,
                                 const uint64_t *__restrict__ flen, const uint32_t *__restrict__ freset,
                                 uint32_t *__restrict__ carry, uint64_t cap, uint64_t *__restrict__ res,
                                 uint64_t *__restrict__ grng, uint64_t *__restrict__ rng, bool unsettled) {
    const bool in = lane < nf;
    const uint32_t valid = in ? (uint32_t)(term != T_NONE ? tpos : flen[lane]) : 0u;
    const uint32_t rst = in ? freset[lane] : 0u;
    const uint64_t errs = __ballot(in && term == T_ERR);
    const uint32_t fe = errs ? (uint32_t)__builtin_ctzll(errs) : nf;  // the walk's last file (or nf)
    // carry[f] = sum of valid over (the last file g < f that resets, f)
    const uint32_t pex = wave_incl_sum(valid) - valid;
    const uint32_t rst_prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rst, 0x138, 0xF, 0xF, false);  // wave_shr:1
    const uint64_t starts = __ballot(lane == 0 || rst_prev != 0);
    const uint64_t le = lane == 63 ? ~0ull : (2ull << lane) - 1;
    const uint32_t g = 63 - (uint32_t)__builtin_clzll(starts & le);
    const uint32_t cf = pex - (uint32_t)__shfl((int)pex, (int)g);
    if (in && lane <= fe) carry[lane] = cf;
    // the file the walk ends with: the error file, else the last
    const uint32_t fl = fe < nf ? fe : nf - 1;
    const uint32_t last_cf = (uint32_t)__shfl((int)cf, (int)fl), last_v = (uint32_t)__shfl((int)valid, (int)fl);
    const uint32_t last_rst = (uint32_t)__shfl((int)rst, (int)fl);
    const uint64_t n_end = nf ? (uint64_t)__shfl((long long)(r0 + nrec), (int)fl) : 0ull;
    if (lane == 0) {
        uint32_t last = 0;
        if (nf) last = last_cf + last_v;
        if (fe < nf) {
            res[0] = GCK_EUNEXPECTED_EOF;  // (res[2], the error's offset: lane fe, below)
            res[1] = fe;
        } else if (nf && last_rst) {
            last = 0;
        }
        res[3] = fe < nf ? fe + 1 : nf;
        res[4] = last;
        res[5] = n_end;
        grng[0] = 0;
        grng[1] = n_end < cap ? n_end : cap;
        if (unsettled) grng[1] = 0;
        rng[0] = 0;
        rng[1] = grng[1];
    }
    if (fe < nf && lane == fe) res[2] = tpos;
}

// Record slots, file summaries and (device path) the run's bookkeeping in one
// launch (four to five launches before, each ~5 us of dispatch for ~1 us of
// work).  Block b of the scan is the b-th wavefront to arrive (a ticket), so
// the single-pass look-back only ever waits on wavefronts that are already
// running: each publishes its block total at once and its inclusive prefix as
// soon as it knows it (lb[b]: value | kLbAgg or kLbInc).  The wavefront that
// finishes last (a second ticket) writes the per-file summaries -- records
// of the file and the terminal condition of its last non-empty chunk -- then,
// with acct set, runs account_run, and leaves lb and the tickets zeroed for
// the next launch.  Per lane 64 consecutive counts, loaded at once (vector
// loads where aligned).  rec_base[n] and *base_out = min(total, cap); a total
// past cap is flagged in *overflow (the exact host path reruns).
constexpr uint64_t kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbVal = kLbAgg - 1;
// the wavefront's block index: arrival order (a ticket)
__device__ __forceinline__ uint32_t lb_ticket(uint32_t *tickets) {
    uint32_t tk = 0;
    if ((threadIdx.x & 63) == 0) tk = atomicAdd(&tickets[0], 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)tk);
}
// block b's exclusive base: its total published at once, then the earlier
// blocks' totals / inclusive prefixes read back until an inclusive one
__device__ uint64_t lookback_excl(uint64_t *lb, uint32_t b, uint64_t btot) {
    const uint32_t lane = threadIdx.x & 63;
    if (b == 0) {
        if (lane == 0) __hip_atomic_store(&lb[0], btot | kLbInc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&lb[b], btot | kLbAgg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // lane k reads block top - k: up to 64 predecessors per round trip
    // (one at a time, a block waited for one L2 round trip per predecessor)
    uint64_t excl = 0;
    for (int64_t top = (int64_t)b - 1; top >= 0;) {
        const int64_t j = top - (int64_t)lane;
        const uint64_t w = j >= 0 ? __hip_atomic_load(&lb[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : kLbInc;  // before block 0: an inclusive prefix of 0
        const uint64_t inc = __ballot((w & kLbInc) != 0), nready = __ballot((w & (kLbAgg | kLbInc)) == 0);
        // the nearest inclusive prefix (lane fi) ends the look-back; every
        // block between must have published its total
        const uint32_t fi = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
        const uint64_t need = fi < 64 ? (2ull << fi) - 1 : ~0ull;
        if (nready & need) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t v = lane <= fi ? (w & kLbVal) : 0;
        // sum over the lanes (values < 2^48: two 24-bit halves)
        const uint64_t sv = lane63(wave_incl_sum64(v));
        excl += sv;
        if (fi < 64) break;
        top -= 64;
    }
    if (lane == 0) __hip_atomic_store(&lb[b], (excl + btot) | kLbInc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}
// true in the wavefront that finishes last (every block's output visible)
__device__ bool lb_last_done(uint32_t *tickets, uint32_t nb) {
    __threadfence();
    uint32_t dn = 0;
    if ((threadIdx.x & 63) == 0) dn = atomicAdd(&tickets[1], 1u);
    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)dn) != nb - 1) return false;
    __threadfence();
    return true;
}
// The device path's validation/fixup rounds 1..kRounds (round 0 is k_walk's),
// run at the head of k_scan_chunks when round 0 found an inconsistent chunk:
// the rounds of k_fixup / k_validate, separated by grid-wide barriers (the
// launch's workgroups are all resident: one wavefront each, a few dozen).
// Without an inconsistency (C3: none) this costs one load; the five launches
// it replaces cost ~25 us per step.  val[r]: round r's inconsistent chunks.
struct Settle {
    const uint8_t *arena;
    const uint64_t *fbase, *flen;
    const uint32_t *ch_file;
    const uint64_t *ch_end;
    uint32_t *ch_bad;
    uint64_t *ch_exit, *ch_wend, *ch_aentry;
    uint2 *s_kv;
    uint32_t cap, chunk_shift;
    uint32_t *val;      // nullptr: no settle rounds (the host path launches them)
    uint32_t *fixups;   // CNT_FIXUP
    uint32_t *bar;      // grid barrier arrivals (zeroed per run)
};
// grid barrier: every wavefront of the launch arrives once per phase
__device__ void grid_sync(uint32_t *bar, uint32_t target) {
    __threadfence();
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(bar, 1u);
        while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence();
}
__device__ void settle_rounds(const Settle &st, uint32_t nc, const uint32_t *f_first_chunk, const uint32_t *f_nchunks,
                              uint64_t *ch_entry, uint32_t *ch_count, uint32_t *ch_term, uint64_t *ch_tpos) {
    const uint32_t lane = threadIdx.x & 63, G = gridDim.x, T = G * 64, t = blockIdx.x * 64 + lane;
    uint32_t phase = 0;
    for (int r = 0; r < kRounds; ++r) {
        if (__hip_atomic_load(&st.val[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) break;  // (the same in every wave)
        for (uint32_t c = t; c < nc; c += T)
            if (st.ch_bad[c])
                fixup_chunk(c, st.arena, st.fbase, st.flen, st.ch_file, st.ch_end, f_first_chunk, f_nchunks, st.ch_bad,
                            ch_entry, ch_count, st.ch_exit, ch_term, ch_tpos, st.ch_wend, st.ch_aentry, st.s_kv, st.cap,
                            st.chunk_shift, st.fixups);
        grid_sync(st.bar, ++phase * G);
        uint32_t nbad = 0;
        for (uint32_t c = t; c < nc; c += T)
            nbad += validate_chunk(c, st.ch_file, st.ch_end, ch_entry, st.ch_exit, ch_term, f_first_chunk, st.ch_bad);
        const uint32_t sum = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(nbad), 63);
        if (lane == 0 && sum) atomicAdd(&st.val[r + 1], sum);
        grid_sync(st.bar, ++phase * G);
    }
}
// workgroups a settling k_scan_chunks launch has at least (one wavefront each)
constexpr uint32_t kSettleBlocks = 64;

__global__ __launch_bounds__(64) void k_scan_chunks(const uint32_t *ch_count, uint64_t *rec_base,
                                                    uint32_t n, uint64_t *lb, uint64_t *base_out, uint64_t cap,
                                                    uint32_t *__restrict__ overflow,
                                                    const uint32_t *__restrict__ f_first_chunk,
                                                    const uint32_t *__restrict__ f_nchunks,
                                                    const uint64_t *ch_entry,
                                                    const uint32_t *ch_term,
                                                    const uint64_t *ch_tpos, uint32_t *f_term,
                                                    uint64_t *f_tpos, uint64_t *f_first_rec, uint64_t *f_nrec,
                                                    uint32_t nfiles, int acct, const uint64_t *__restrict__ flen,
                                                    const uint32_t *__restrict__ freset, uint32_t *carry,
                                                    uint64_t *res, uint64_t *grng, uint64_t *rng, uint32_t nb, Settle st) {
    static_assert(kScanBlock == 64 * 64, "a lane owns 64 counts");
    if (st.val && __hip_atomic_load(&st.val[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
        settle_rounds(st, n, f_first_chunk, f_nchunks, const_cast<uint64_t *>(ch_entry), const_cast<uint32_t *>(ch_count),
                      const_cast<uint32_t *>(ch_term), const_cast<uint64_t *>(ch_tpos));
    if (blockIdx.x >= nb) return;  // (settle-only workgroups)
    const uint32_t lane = threadIdx.x;
    uint32_t *tickets = reinterpret_cast<uint32_t *>(lb + nb);
    const uint32_t b = lb_ticket(tickets);
    const uint32_t i0 = b * kScanBlock + lane * 64;
    uint32_t v[64];
    const bool vec_in = i0 + 64 <= n && (reinterpret_cast<uintptr_t>(ch_count + i0) & 15) == 0;
    if (vec_in) {
        const uint4 *src = reinterpret_cast<const uint4 *>(ch_count + i0);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint4 x = src[k];
            v[4 * k] = x.x;
            v[4 * k + 1] = x.y;
            v[4 * k + 2] = x.z;
            v[4 * k + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 64; ++k) v[k] = i0 + k < n ? ch_count[i0 + k] : 0u;
    }
    uint64_t tot = 0;
#pragma unroll
    for (int k = 0; k < 64; ++k) tot += v[k];
    const uint64_t inc = wave_incl_sum64(tot);
    const uint64_t btot = lane63(inc);
    const uint64_t excl = lookback_excl(lb, b, btot);
    uint64_t run = excl + inc - tot;  // this lane's first base
    const bool vec_out = i0 + 64 <= n && (reinterpret_cast<uintptr_t>(rec_base + i0) & 15) == 0;
    if (vec_out) {
        u32x4 *dst = reinterpret_cast<u32x4 *>(rec_base + i0);
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const uint64_t a = run, c2 = run + v[2 * k];
            run = c2 + v[2 * k + 1];
            u32x4 o;
            o.x = (uint32_t)a;
            o.y = (uint32_t)(a >> 32);
            o.z = (uint32_t)c2;
            o.w = (uint32_t)(c2 >> 32);
            dst[k] = o;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            if (i0 + k < n) rec_base[i0 + k] = run;
            run += v[k];
        }
    }
    if (b == nb - 1 && lane == 0) {
        // past the record-table capacity the range is clamped (later kernels
        // stay in bounds) and the run is flagged for the exact synchronous path
        const uint64_t total = excl + btot;
        if (total > cap) atomicAdd(overflow, 1u);
        rec_base[n] = min(total, cap);
        *base_out = min(total, cap);
    }
    // the last wavefront to finish sees every block's bases
    if (!lb_last_done(tickets, nb)) return;
    uint32_t term = T_NONE;  // lane f's file (the first 64 files)
    uint64_t tpos = 0, r0 = 0, nrec = 0;
    for (uint32_t f = lane; f < nfiles; f += 64) {
        const uint32_t fc = f_first_chunk[f], nc = f_nchunks[f];
        r0 = rec_base[fc];
        nrec = rec_base[fc + nc] - r0;
        f_first_rec[f] = r0;
        f_nrec[f] = nrec;
        term = T_NONE;
        tpos = 0;
        // the terminal chunk is the last non-empty chunk of the file
        for (int64_t k = (int64_t)fc + nc - 1; k >= (int64_t)fc; --k) {
            if (ch_entry[k] != kNone) {
                term = ch_term[k];
                tpos = ch_tpos[k];
                break;
            }
        }
        f_term[f] = term;
        f_tpos[f] = tpos;
    }
    for (uint32_t k = lane; k < nb + 1; k += 64) lb[k] = 0;  // lb and both tickets
    if (!acct) return;
    const bool unsettled =
        st.val && __hip_atomic_load(&st.val[kRounds], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (nfiles <= 64) {
        account_run_wave(nfiles, lane, term, tpos, r0, nrec, flen, freset, carry, cap, res, grng, rng, unsettled);
        return;
    }
    __threadfence();
    __builtin_amdgcn_wave_barrier();
    if (lane == 0)
        account_run(nfiles, flen, freset, f_term, f_tpos, f_first_rec, f_nrec, carry, cap, res, grng, rng,
                    unsettled);
}

// Key offsets of a run's records for the key blob gck_replay returns with
// GCK_OPT_KEYS: koff[i] = the key bytes of records before i (a record's key
// is key_len bytes at its header + 16, a tombstone's included: KeySize 0,
// the key is its "value", core/db.go:151-155), koff[n] = the total.  The same
// single-pass look-back as k_scan_chunks (lb: its own zeroed words).
__global__ __launch_bounds__(64) void k_scan_keys(const uint2 *__restrict__ rec_kv, uint64_t n,
                                                  uint64_t *__restrict__ koff, uint64_t *lb) {
    const uint32_t lane = threadIdx.x, nb = gridDim.x;
    uint32_t *tickets = reinterpret_cast<uint32_t *>(lb + nb);
    const uint32_t b = lb_ticket(tickets);
    const uint64_t i0 = (uint64_t)b * kScanBlock + lane * 64;
    uint32_t v[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) {
        const uint2 kv = i0 + k < n ? rec_kv[i0 + k] : make_uint2(0u, 0u);
        v[k] = kv.x ? kv.x : kv.y;
    }
    uint64_t tot = 0;
#pragma unroll
    for (int k = 0; k < 64; ++k) tot += v[k];
    const uint64_t inc = wave_incl_sum64(tot);
    const uint64_t btot = lane63(inc);
    const uint64_t excl = lookback_excl(lb, b, btot);
    uint64_t run = excl + inc - tot;
#pragma unroll
    for (int k = 0; k < 64; ++k) {
        if (i0 + k < n) koff[i0 + k] = run;
        run += v[k];
    }
    if (b == nb - 1 && lane == 0) koff[n] = excl + btot;
    if (!lb_last_done(tickets, nb)) return;
    for (uint32_t k = lane; k < nb + 1; k += 64) lb[k] = 0;  // lb and both tickets
}

// The same offsets for the entries of a keydir merge (gck_kd_merge's d_mhdr):
// the key bytes of entries [0, n) back to back, the GCK_OPT_KEYS blob of a
// live or multi replay (merged_out).
__global__ __launch_bounds__(64) void k_mo_scan(const gck_kd_entry *__restrict__ E, uint64_t n,
                                                uint64_t *__restrict__ koff, uint64_t *lb) {
    const uint32_t lane = threadIdx.x, nb = gridDim.x;
    uint32_t *tickets = reinterpret_cast<uint32_t *>(lb + nb);
    const uint32_t b = lb_ticket(tickets);
    const uint64_t i0 = (uint64_t)b * kScanBlock + lane * 64;
    uint32_t v[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) v[k] = i0 + k < n ? E[i0 + k].key_len : 0u;
    uint64_t tot = 0;
#pragma unroll
    for (int k = 0; k < 64; ++k) tot += v[k];
    const uint64_t inc = wave_incl_sum64(tot);
    const uint64_t btot = lane63(inc);
    const uint64_t excl = lookback_excl(lb, b, btot);
    uint64_t run = excl + inc - tot;
#pragma unroll
    for (int k = 0; k < 64; ++k) {
        if (i0 + k < n) koff[i0 + k] = run;
        run += v[k];
    }
    if (b == nb - 1 && lane == 0) koff[n] = excl + btot;
    if (!lb_last_done(tickets, nb)) return;
    for (uint32_t k = lane; k < nb + 1; k += 64) lb[k] = 0;  // lb and both tickets
}
// recs[i] = entry i's record; with keys, its key bytes (K + key_off, zero
// padded to 8 B) at keys + koff[i], unpadded
__global__ void k_mo_out(const gck_kd_entry *__restrict__ E, const uint8_t *__restrict__ K,
                         const uint64_t *__restrict__ koff, uint64_t n, gck_rec *__restrict__ recs,
                         uint8_t *__restrict__ keys) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        recs[i] = E[i].rec;
        if (!keys) continue;
        const uint32_t len = E[i].key_len;
        const uint8_t *src = K + E[i].key_off;
        uint8_t *dst = keys + koff[i];
        uint32_t j = 0;
        if ((reinterpret_cast<uintptr_t>(dst) & 3) == 0)  // (src is 8-byte aligned)
            for (; j + 4 <= len; j += 4)
                *reinterpret_cast<uint32_t *>(dst + j) = *reinterpret_cast<const uint32_t *>(src + j);
        for (; j < len; ++j) dst[j] = src[j];
    }
}

// The key bytes of records [0, n) back to back (koff from k_scan_keys): a lane
// per record, dwords where source and destination allow, else bytes.
__global__ void k_gather_keys(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ rec_off,
                              const uint2 *__restrict__ rec_kv, const uint64_t *__restrict__ koff, uint64_t n,
                              uint8_t *__restrict__ blob) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint2 kv = rec_kv[r];
        const uint32_t len = kv.x ? kv.x : kv.y;
        const uint8_t *src = arena + rec_off[r] + 16;
        uint8_t *dst = blob + koff[r];
        uint32_t i = 0;
        if (((reinterpret_cast<uintptr_t>(src) ^ reinterpret_cast<uintptr_t>(dst)) & 3) == 0) {
            for (; i < len && (reinterpret_cast<uintptr_t>(src + i) & 3); ++i) dst[i] = src[i];
            for (; i + 4 <= len; i += 4)
                *reinterpret_cast<uint32_t *>(dst + i) = *reinterpret_cast<const uint32_t *>(src + i);
        }
        for (; i < len; ++i) dst[i] = src[i];
    }
}

// row_first[row] = the first record whose value ends after the row's first
// byte.  Record r sets the rows from its start to its end, [ceil(rs / 4 KiB),
// ceil(ve / 4 KiB)); k_row_tail sets the rows after a file's last record.
// Record r = [rs, ve) is the first record ending past the start of every row
// block (kBlkBytes = 64 rows) that starts inside it.
#ifndef GCK_BLOCK_ROWS
#define GCK_BLOCK_ROWS 64
#endif
constexpr int kBlockRows = GCK_BLOCK_ROWS;  // rows per k_crc_rows work item (a "row block"): 32 or 64
static_assert(kBlockRows == 32 || kBlockRows == 64, "k_crc_rows: a lane per row of the block");
constexpr int kNibDw = kBlockRows / 8;      // nibble dwords per lane (8 rows of 4 blocks each)
constexpr uint64_t kBlkBytes = (uint64_t)kBlockRows * kRow;
__device__ __forceinline__ void set_blk_first(uint32_t *blk_first, uint64_t r, uint64_t rs, uint64_t ve) {
    for (uint64_t q = (rs + kBlkBytes - 1) / kBlkBytes; q < (ve + kBlkBytes - 1) / kBlkBytes; ++q)
        blk_first[q] = (uint32_t)r;
}

struct DirectEmit {
    uint64_t *rec_off;
    uint2 *rec_kv;
    uint32_t *rec_file;
    uint32_t *blk_first;
    uint64_t rb, n_total, base;
    uint32_t f, re;
    __device__ void operator()(uint32_t i, uint64_t p, const Hdr &h) const {
        const uint64_t r = rb + i;
        if (r < n_total) {
            rec_off[r] = base + p;
            rec_kv[r] = make_uint2(h.ks, h.vs);
            rec_file[r] = f;
        }
        set_blk_first(blk_first, r < n_total ? r : re, base + p, base + p + 16 + (uint64_t)h.ks + h.vs);
    }
    __device__ void prime() const {}
};

// Record table in walk order and the row index row_first, in one launch.
//
// Records: a wavefront per kCompactChunks consecutive chunks c0 + c (the
// chunk arrays are passed offset by c0; the stage is indexed by global chunk)
// copies their staged (KeySize, ValueSize) pairs and rebuilds the record
// offsets from each chunk's entry (an arena offset, left by the walk) by a
// scan of the entry sizes; chunks that overflowed the stage re-walk straight
// into the table.  Every load a chunk needs -- count, record base, file,
// entry and the first kPreBatches batches of its stage -- is issued for all of
// the wavefront's chunks before the first is written: one round trip per
// wavefront instead of two per chunk (the file's base was a second, dependent
// one), and a quarter of the wavefronts (the grid ran in eight rounds of
// resident wavefronts, each paying its round trips).  The stage interleaves
// slot i of kStageIl consecutive chunks, so a workgroup's stage lines are
// fetched once per CU.
//
// row_first[row] = the first record whose value ends after the row's first
// byte; every row gets exactly one write: record r sets the rows from its start
// to its end, [ceil(rs / 4 KiB), ceil(ve / 4 KiB)) -- to r, or to the range end
// re = rng[1] for a record past the table (r >= n_total); the rows after file
// f's last record (its length, or where its walk stopped: EOF class or startup
// error), up to the next file's first row, get min(ffirst[f] + fnrec[f], re)
// (wavefront w takes files w, w + W, ...); row n_rows (the sentinel) gets re.
// (Three launches before: k_row_fill set every row to re first, k_row_tail
// the tails; 12 us and a 33 MB pre-fill per C3 step.)
#ifndef GCK_COMPACT_CHUNKS
#define GCK_COMPACT_CHUNKS 1
#endif
constexpr uint32_t kCompactChunks = GCK_COMPACT_CHUNKS;
struct RowTails {
    const uint32_t *fterm;
    const uint64_t *ftpos, *ffirst, *fnrec, *rng;
    uint32_t nfiles;
    uint64_t n_rows, n_blocks;  // n_blocks = ceil(n_rows / 64): blk_first has n_blocks + 1 entries
    const uint32_t *unsettled;  // device path: the last settle round's count (nonzero: rows all 0, no table)
};
__global__ __launch_bounds__(1024) void k_compact(const uint8_t *__restrict__ arena,
                                                  const uint64_t *__restrict__ fbase,
                                                  const uint64_t *__restrict__ flen,
                                                  const uint32_t *__restrict__ ch_file,
                                                  const uint64_t *__restrict__ ch_wend,
                                                  const uint64_t *__restrict__ ch_entry,
                                                  const uint64_t *__restrict__ ch_aentry,
                                                  const uint32_t *__restrict__ ch_count,
                                                  const uint64_t *__restrict__ rec_base,
                                                  const uint2 *__restrict__ s_kv, uint32_t cap, uint32_t c0,
                                                  uint32_t n_chunks, uint64_t n_total, uint64_t *rec_off,
                                                  uint2 *rec_kv, uint32_t *rec_file, uint32_t *blk_first,
                                                  uint32_t *counters, RowTails rt) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = blockIdx.x * 16 + (threadIdx.x >> 6), cw = wv * kCompactChunks;
    const uint32_t re = (uint32_t)rt.rng[1];
    if (rt.unsettled && *rt.unsettled) {
        // chunks left inconsistent (the run is redone on the host path): the
        // walks may leave rows unset, so every row points at record 0 and
        // k_crc_rows finds no record end (finalize's range is empty)
        for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= rt.n_blocks;
             q += (uint64_t)gridDim.x * blockDim.x)
            blk_first[q] = 0;
        return;
    }
    GCK_CLK_BEGIN();
    if (cw < n_chunks) {
        constexpr uint32_t K = kCompactChunks;
        uint32_t cnt[K], f[K];
        uint64_t rb[K], ae[K];
        uint2 pre[K][kPreBatches];
#pragma unroll
        for (uint32_t j = 0; j < K; ++j) {
            const uint32_t c = min(cw + j, n_chunks - 1);  // (a chunk past the end repeats the last: skipped below)
            cnt[j] = ch_count[c];
            rb[j] = rec_base[c];
            f[j] = ch_file[c];
            ae[j] = ch_aentry[c];
#pragma unroll
            for (uint32_t k = 0; k < kPreBatches; ++k) pre[j][k] = s_kv[stage_slot(c0 + c, 64 * k + lane, cap)];
        }
#pragma unroll
        for (uint32_t j = 0; j < K; ++j) {
            const uint32_t c = cw + j;
            // no entry (count 0): nothing staged
            if (c >= n_chunks || cnt[j] == 0) continue;
            if (cnt[j] <= cap) {
                uint64_t run = ae[j];  // arena offset of the next record
                // batches past the preloaded ones: the next batch's stage entries
                // are loaded while this batch is written
                uint2 nxt = make_uint2(0u, 0u);
                for (uint32_t i0 = 0; i0 < cnt[j]; i0 += 64) {
                    const uint32_t i = i0 + lane;
                    const bool in = i < cnt[j];
                    const uint32_t b = i0 / 64;  // (uniform)
                    uint2 kv = nxt;
#pragma unroll
                    for (uint32_t k = 0; k < kPreBatches; ++k)
                        if (b == k) kv = pre[j][k];
                    if (!in) kv = make_uint2(0u, 0u);
                    if (b + 1 >= kPreBatches)
                        nxt = i + 64 < cnt[j] ? s_kv[stage_slot(c0 + c, i + 64, cap)] : make_uint2(0u, 0u);
                    // entry size (a tombstone's: 16 + len(key), as KeySize = 0); the
                    // inclusive scan is exact in 24-bit halves (entries < 2^33)
                    const uint64_t e = in ? 16ull + kv.x + kv.y : 0ull;
                    const uint32_t lo = wave_incl_sum((uint32_t)(e & 0xFFFFFFu)), hi = wave_incl_sum((uint32_t)(e >> 24));
                    const uint64_t r = rb[j] + i;
                    if (in) {
                        const uint64_t ve = run + (((uint64_t)hi << 24) + lo);
                        if (r < n_total) {
                            rec_off[r] = ve - e;
                            rec_kv[r] = kv;
                            rec_file[r] = f[j];
                        }
                        set_blk_first(blk_first, r < n_total ? r : re, ve - e, ve);
                    }
                    run += ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 24) +
                           (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
                }
            } else if (lane == 0) {
                atomicAdd(&counters[CNT_STAGE], 1u);
                const uint64_t base = fbase[f[j]];
                DirectEmit em{rec_off, rec_kv, rec_file, blk_first, rb[j], n_total, base, f[j], re};
                uint32_t count, term;
                uint64_t exit, tpos;
                walk_chain(arena, base, flen[f[j]], ch_wend[c], ch_entry[c], em, count, exit, term, tpos);
            }
        }
    }
    // the blocks that start after each file's last record (up to the next
    // file's first row), and the sentinel
    const uint32_t W = gridDim.x * 16;
    for (uint32_t f = wv; f < rt.nfiles; f += W) {
        const uint64_t end = fbase[f] + (rt.fterm[f] != T_NONE ? rt.ftpos[f] : flen[f]);
        const uint64_t r1 = f + 1 < rt.nfiles ? fbase[f + 1] / kRow : rt.n_rows;  // rows < r1
        const uint32_t v = (uint32_t)min(rt.ffirst[f] + rt.fnrec[f], (uint64_t)re);
        for (uint64_t q = (end + kBlkBytes - 1) / kBlkBytes + lane; q < (r1 + kBlockRows - 1) / kBlockRows; q += 64)
            blk_first[q] = v;
    }
    if (wv == 0 && lane == 0) blk_first[rt.n_blocks] = re;
    GCK_CLK_END(4, cw / kCompactChunks);
}

__device__ __forceinline__ uint64_t value_end(const uint64_t *rec_off, const uint2 *rec_kv, uint64_t r) {
    const uint2 kv = rec_kv[r];
    return rec_off[r] + 16 + (uint64_t)kv.x + kv.y;  // tombstone: KeySize 0, the key is the "value"
}

constexpr int kArenaAux = 2;     // k_crc_rows' arena loads: non-temporal (buffer aux bit; DESIGN.md §6 load policy)
#ifndef GCK_CLAIM
#define GCK_CLAIM 1
#endif
constexpr uint32_t kClaim = GCK_CLAIM;   // consecutive row blocks per k_crc_rows queue claim
#ifndef GCK_LATE_CLAIM
#define GCK_LATE_CLAIM 13
#endif
// where in a block k_crc_rows claims the block after next, in 16ths of the
// block's quads (-1: at the block's start).  Claiming one block, late, holds
// a wave's look-ahead to ~1.2 blocks instead of up to 3 when the queue runs
// dry: the kernel's tail (wave-end spread) shrinks, -0.04 ms at C3
// (profiles/r5f).  (The claim must fall inside the block, whatever its quad
// count: a block without one re-processed block 0 forever.)
constexpr int kLateClaim = GCK_LATE_CLAIM;
static_assert(kLateClaim < 16, "the late claim lies inside the block");
#ifndef GCK_STATIC_EIGHTHS
#define GCK_STATIC_EIGHTHS 4
#endif
constexpr uint32_t kStaticEighths = GCK_STATIC_EIGHTHS;     // eighths of k_crc_rows' full rounds assigned statically
constexpr uint64_t kEpScratch = 256 * 64;  // (c, pre) scratch slots past the records (k_crc_rows)
#ifdef GCK_XP_EBLK
constexpr uint64_t kEpBytes = 24;  // (c, pre) + the end block
#else
constexpr uint64_t kEpBytes = 8;
#endif

#ifdef GCK_CLOCK_STAMPS
// the plain non-temporal stream read (diag.hip's k_stream_read<true>), stamped
__global__ __launch_bounds__(256) void k_clk_stream(const uint4 *__restrict__ p, uint64_t n16, uint32_t *sink) {
    GCK_CLK_BEGIN();
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
    uint32_t acc = 0;
    auto ld = [&](uint64_t i) {
        const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p + i));
        return v.x ^ v.y ^ v.z ^ v.w;
    };
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x * 4 + threadIdx.x; i < n16; i += stride) {
        const uint32_t a = ld(i), b = i + 256 < n16 ? ld(i + 256) : 0u, c = i + 512 < n16 ? ld(i + 512) : 0u,
                       d = i + 768 < n16 ? ld(i + 768) : 0u;
        acc ^= a ^ b ^ c ^ d;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
    GCK_CLK_END(1, blockIdx.x * 4 + (threadIdx.x >> 6));
}
#endif

template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWMASK, 0xF, false);
}

// LDS image of the CRC tables (identical in every k_crc_rows workgroup).
__device__ __forceinline__ void fill_crc_lds(uint32_t *lds, const uint32_t *__restrict__ g_slice,
                                             const uint32_t *__restrict__ g_nib) {
    fill_slice_lds(lds, g_slice);
    // lane-shift tables: nibble q (from bit 0 of G), value v, lane l at byte
    // 4 kNibBase + 4096 q + 256 v + 4 l (every lane on its own bank); the
    // lookup address is one v_perm_b32 (see k_crc_rows)
    for (uint32_t i = threadIdx.x; i < 8192; i += blockDim.x) {
        const uint32_t l = i & 63, v = (i >> 6) & 15, q = i >> 10;
        lds[kNibBase + i] = g_nib[(l * 8 + q) * 16 + v];
    }
    __syncthreads();
}

// The HBM-bound kernel.  A wavefront owns a 4 KiB row; lane k owns slab k =
// bytes [64k, 64k+64).  Branch-free: every lane runs one CRC register from 0
// over its 16 words (slicing-by-4, LDS tables) and keeps the register at each
// 16 B block start (c1, c2, c3 after words 3, 7, 11; c0 = 0) and at the slab
// end, G = F(0, slab).  Record boundaries never enter the arithmetic:
//   - G is referenced to the row end, Z_{64(63-k)}(G) (8 nibble lookups in the
//     lane's LDS table), and an inclusive prefix XOR over the wave (DPP) gives
//     rrow = F(0, row) (lane 63) and, per lane, pre = the exclusive prefix =
//     the slabs before k referenced to the row end;
//   - per record end in block b of slab k the lane stores (c_b, pre) at the
//     record's slot; k_finalize continues c_b over the <= 16 bytes of the
//     block up to the record end and stitches rows (see there).
// Outputs: out_ep (c, pre) per record, out_rend per row (rrow).
//
// Work: row blocks of 64 consecutive rows, the first half of the full rounds
// static, the rest from an atomic queue (late-starting or slow wavefronts take
// fewer).  Per block the record ends of its rows (records [row_first[first
// row], row_first[first row + 64]), in offset order) become per-lane nibbles
// (bit b of row j's nibble in lane k: a record's last byte lies in block b of
// slab k); the first 64 ends are loaded one block ahead.  The block's 64 rrow
// values leave in one coalesced store, so per row the vector-memory queue
// holds only the 4 x 16 B row loads and one 8 B (c, pre) store.  Rows are
// local to the launch: arena, row_first and out_rend point at its first row
// (row0 in the whole arena); n_total is the record-slot scratch base (64
// slots per wavefront), rend_scratch 64 row slots.
//
// Memory pipeline: the row data are buffer loads (row base in a scalar
// resource, lane offset in a fixed VGPR) issued one row ahead.  No scalar
// loads in the loop: an outstanding SMEM load would make every LDS wait
// (lgkmcnt(0)) wait for HBM too.  Every lane stores on every path (lanes
// without a record end to an out-of-range offset, dropped), so the compiler's
// vmcnt waits count the same stores on every path and stay a row behind the
// loads.
//
// Codegen is part of the design here: this text compiles to round 2's
// instruction stream (register arrays of one row, select-form captures, each
// row's store before the next row's loads).  Round 3 rewrote it with scalar
// registers and mask-form captures: the same work, the stores sunk behind the
// next row's loads, and a tail of late wavefronts (clock stamps: last wave
// 0.6 ms after the median against 0.13 now): 5.45-5.56 against 5.18-5.20 ms on
// one box (profiles/r4f/ab_r2_head_port.log, profiles/r4a/bisect_r3_commits.log).
// Compare the ISA (hipcc --cuda-device-only -S) before and after any edit.
#ifndef GCK_PREFETCH
#define GCK_PREFETCH 1
#endif
constexpr int kPrefetch = GCK_PREFETCH;  // steps between a row's loads and its processing (2, 3 measured slower)
__global__ __launch_bounds__(1024) void k_crc_rows(const uint8_t *__restrict__ arena, uint64_t n_rows,
                                                   const uint32_t *__restrict__ blk_first, uint64_t n_total,
                                                   const uint32_t *__restrict__ g_slice,
                                                   const uint32_t *__restrict__ g_nib, uint2 *__restrict__ out_ep,
                                                   uint32_t *__restrict__ out_rend,
                                                   uint32_t *__restrict__ rend_scratch,
                                                   uint32_t *__restrict__ queue,
                                                   const uint64_t *__restrict__ rec_off,
                                                   const uint2 *__restrict__ rec_kv, uint64_t row0
#ifdef GCK_XP_EBLK
                                                   , uint8_t *__restrict__ out_blk
#endif
                                                   ) {
    constexpr int NR = 1;                     // rows per step (two measured slower: 5.70 vs 5.64 ms)
    constexpr int kSteps = kBlockRows / NR;  // steps per block
    constexpr int kLateQd = kLateClaim < 0 ? -1 : kLateClaim * (kSteps / 4) / 16;  // the claim's quad
    __shared__ uint32_t lds[40960];  // 128 KiB slicing tables x32 copies + 32 KiB lane-shift tables
    fill_crc_lds(lds, g_slice, g_nib);
    const uint32_t lane = threadIdx.x & 63, l31 = lane & 31;
    static_assert(kNibBase * 4 == 0x20000, "shift-table addresses: byte 2 of the v_perm base");
    const uint32_t nbase = kNibBase * 4 + lane * 4;  // byte 0: the lane's bank, byte 2: the region
    const uint32_t lb0 = l31 * 4, lb1 = 65536 + l31 * 4;
    // load k of a row: lane p + 16 b reads the 16 B at 1024 k + 64 p + 16 b,
    // so each load instruction is one contiguous KiB of the row (whole cache
    // lines, which the non-temporal hint needs); two permlane swap stages then
    // give lane L the four blocks of its slab [64 L, 64 L + 64)
    const uint32_t s_rel = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint64_t n_blocks = (n_rows + kBlockRows - 1) / kBlockRows;
    // (c, pre) stores go through a buffer resource based at the block's first
    // record: lanes without a record end store at an out-of-range offset, which
    // the bounds check drops (no traffic), while every lane still issues the
    // store (a fixed count for the compiler's vmcnt waits)
    constexpr uint32_t kDrop = 0xFFFFFFF0u;
    __amdgpu_buffer_rsrc_t ep_rsrc = make_rsrc(out_ep, 0x7FFFFFF0);
    uint32_t ra0 = 0;
    auto store_ep = [&](uint32_t off, uint32_t cv, uint32_t pv) {
        u32x2 v;
        v.x = cv;
        v.y = pv;
        __builtin_amdgcn_raw_buffer_store_b64(v, ep_rsrc, (int)off, 0, 0);
    };
#ifdef GCK_XP_EBLK
    // experiment: each record end's 16 B block beside its (c, pre)
    __amdgpu_buffer_rsrc_t blk_rsrc = make_rsrc(out_blk, 0x7FFFFFF0);
    auto store_blk = [&](uint32_t off8, const u32x4 &v) {
        __builtin_amdgcn_raw_buffer_store_b128(v, blk_rsrc, (int)(off8 == kDrop ? kDrop : off8 * 2u), 0, 0);
    };
#define GCK_PICK_BLK(wv, b)                                                                          \
    u32x4 {(b) == 0 ? wv[0] : (b) == 1 ? wv[4] : (b) == 2 ? wv[8] : wv[12],                          \
           (b) == 0 ? wv[1] : (b) == 1 ? wv[5] : (b) == 2 ? wv[9] : wv[13],                          \
           (b) == 0 ? wv[2] : (b) == 1 ? wv[6] : (b) == 2 ? wv[10] : wv[14],                         \
           (b) == 0 ? wv[3] : (b) == 1 ? wv[7] : (b) == 2 ? wv[11] : wv[15]}
#endif

    // Work assignment: the first rounds are static (wavefront w of W takes
    // blocks k W + w, k < n_static: every wavefront streams its share with no
    // claims), the rest come from an atomic queue kClaim blocks at a time
    // (late or slow wavefronts take fewer).  Measured without compute, the
    // static order streams 0.3 ms faster over C3 than the queue alone; with
    // compute, a fully static split loses to the queue's balance (6.02 vs
    // 5.82 ms), half static / half queue is best (5.77).
    const uint32_t W = gridDim.x * kWaves, w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWaves + (threadIdx.x >> 6)));
    const uint32_t n_static = (uint32_t)(n_blocks / W) * kStaticEighths / 8;
    uint32_t st_k = 0;
    uint32_t last = kClaim - 1;
    auto grab = [&]() -> uint32_t {  // next block index
        if (st_k < n_static) return (st_k++) * W + w;
        if (last % kClaim == kClaim - 1) {
            uint32_t v = 0;
            if (lane == 0) v = atomicAdd(queue, 1u);
            last = n_static * W + kClaim * (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
        } else {
            ++last;
        }
        return last;
    };
    struct Plan {
        uint32_t ra;  // the block's first record end (every lane: a vector load, no SMEM in the loop)
        uint32_t re;  // the next block's
    };
    auto load_plan = [&](uint64_t q, Plan &p) {
        const uint64_t qc = q < n_blocks ? q : n_blocks - 1;
        p.re = blk_first[qc + 1];
        p.ra = blk_first[qc];
    };
    // The block's nibbles from its record ends (records [ra0, re) end in its
    // rows, in offset order): a lane per record computes (row, slab, block) of
    // its last byte, then a uniform loop hands each end to the slab's lane
    // (nibble dword chosen by a uniform index).  The first 64 record ends of a
    // block are loaded one block ahead (Batch); later ones (blocks with more
    // than 64 ends) on the spot.
    struct Batch {
        uint64_t off;
        uint2 kv;
    };
    auto load_batch = [&](const Plan &p, Batch &b) {
        const uint32_t r = min((uint32_t)__builtin_amdgcn_readlane((int)p.ra, 0) + lane, (uint32_t)(n_total - 1));
        b.off = rec_off[r];
        b.kv = rec_kv[r];
    };
    auto build_nibs = [&](uint64_t row_b, uint32_t ra0_, uint32_t re_, const Batch *first, uint32_t (&nb)[kNibDw]) {
#pragma unroll
        for (int d = 0; d < kNibDw; ++d) nb[d] = 0;
        const uint64_t base = (row0 + row_b) * kRow;
        for (uint32_t b0 = ra0_; b0 < re_; b0 += 64) {
            const uint32_t r = b0 + lane;
            uint32_t code = 0;
            if (r < re_) {
                const uint64_t end = first && b0 == ra0_ ? first->off + 16 + (uint64_t)first->kv.x + first->kv.y
                                                         : value_end(rec_off, rec_kv, r);
                const uint64_t rel = end - 1 - base;  // < 64 rows
                code = ((uint32_t)(rel >> 12) << 8) | ((uint32_t)(rel >> 6) & 63u) << 2 | ((uint32_t)(rel >> 4) & 3u);
            }
            // ends in offset order, so each nibble dword's ends are a run:
            // per dword d a uniform loop over its ends (static register index).
            // Target lane and bit decoded by every lane at once; the loop only
            // reads them (two readlanes) and ORs the bit into lane k.
            const uint32_t dd = r < re_ ? code >> 11 : 8u;
            const uint32_t tk = (code >> 2) & 63u, tbit = (1u << (code & 3u)) << (4 * ((code >> 8) & 7u));
#pragma unroll
            for (int d = 0; d < kNibDw; ++d) {
                uint64_t act = __ballot(dd == (uint32_t)d);
                while (act) {
                    const int i = __builtin_ctzll(act);
                    act ^= 1ull << i;
                    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)tk, i);
                    const uint32_t bit = (uint32_t)__builtin_amdgcn_readlane((int)tbit, i);
                    nb[d] |= lane == k ? bit : 0u;
                }
            }
        }
    };
    struct RowBuf {
        u32x4 x[4];
    };
    auto issue = [&](uint64_t row0, RowBuf (&bs)[NR]) {
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            // 32-bit row index (rows < 2^32): the clamp stays on the scalar unit
            const uint32_t r = min((uint32_t)(row0 + i), (uint32_t)(n_rows - 1));
            const __amdgpu_buffer_rsrc_t rrow = make_rsrc(arena + (uint64_t)r * kRow, kRow);
#pragma unroll
            for (int k = 0; k < 4; ++k) bs[i].x[k] = __builtin_amdgcn_raw_buffer_load_b128(rrow, s_rel + 1024 * k, 0, kArenaAux);
        }
    };
    // one step: rows row0 .. row0+NR-1 = rows j0 .. j0+NR-1 of the block;
    // nib holds their plan nibbles from bit 0 up
    auto process = [&](uint64_t row0, uint32_t j0, uint32_t nib, uint32_t &rel, const RowBuf (&bs)[NR],
                       uint32_t &rend_buf) {
        uint32_t w[NR][16];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            // w[i][4 k + c] = dword c of load k; M[b][k] = lane (p + 16 b)'s load k
            // (= row bytes 1024 k + 64 p + 16 b).  permlane32_swap on (k, k+2)
            // then permlane16_swap on (k, k+1) transpose M over each lane group
            // {p, p+16, p+32, p+48}: lane p + 16 r ends with M[0..3][r] = the
            // bytes 1024 r + 64 p + 16 b, b = 0..3, i.e. slab 16 r + p.
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                w[i][4 * k] = bs[i].x[k].x;
                w[i][4 * k + 1] = bs[i].x[k].y;
                w[i][4 * k + 2] = bs[i].x[k].z;
                w[i][4 * k + 3] = bs[i].x[k].w;
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const auto r = __builtin_amdgcn_permlane32_swap(w[i][4 * k + c], w[i][4 * (k + 2) + c], false, false);
                    w[i][4 * k + c] = r[0];
                    w[i][4 * (k + 2) + c] = r[1];
                }
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
#pragma unroll
                for (int k = 0; k < 4; k += 2) {
                    const auto r = __builtin_amdgcn_permlane16_swap(w[i][4 * k + c], w[i][4 * (k + 1) + c], false, false);
                    w[i][4 * k + c] = r[0];
                    w[i][4 * (k + 1) + c] = r[1];
                }
            }
        }
        // NR independent chains interleaved: NR table reads in flight per step
        uint32_t a[NR], c1[NR], c2[NR], c3[NR], G[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) a[i] = w[i][0];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
#pragma unroll
            for (int i = 0; i < NR; ++i) {
                const uint32_t nx = j < 15 ? w[i][j < 15 ? j + 1 : 15] : 0u;
                if (j == 15) {
                    G[i] = slice4x(lds, lb0, lb1, a[i], 0u);
                } else if ((j & 3) == 3) {
                    const uint32_t c = slice4x(lds, lb0, lb1, a[i], 0u);
                    if (j == 3) c1[i] = c;
                    if (j == 7) c2[i] = c;
                    if (j == 11) c3[i] = c;
                    a[i] = c ^ nx;
                } else {
                    a[i] = slice4x(lds, lb0, lb1, a[i], nx);
                }
            }
        }
        // Z_{64(63-lane)}(G) of every row (8 nibble lookups in the lane's
        // table), then the NR wave scans interleaved so each DPP read finds
        // its source written a few instructions earlier (no s_nop hazards).
        // Lookup addresses: byte k of ge / go holds nibble 2k / 2k+1 of G
        // with the nibble's index in its high half, which makes byte 1 of the
        // address (table q, entry v): one v_perm_b32 per lookup, 3 VALU to
        // split G (was a shift, an and and an add per lookup)
        uint32_t P[NR], pre[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            // (x & m) | q in one v_bitop3_b32 (truth table 0xEA; the two
            // constants live in registers set up outside the loop)
            const uint32_t ge = __builtin_amdgcn_bitop3_b32(G[i], 0x0F0F0F0Fu, 0x60402000u, 0xEA);
            const uint32_t go = __builtin_amdgcn_bitop3_b32(G[i] >> 4, 0x0F0F0F0Fu, 0x70503010u, 0xEA);
            uint32_t t[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                t[2 * k] = lds_at(lds, __builtin_amdgcn_perm(ge, nbase, 0x0C020000u | ((4u + k) << 8)));
                t[2 * k + 1] = lds_at(lds, __builtin_amdgcn_perm(go, nbase, 0x0C020000u | ((4u + k) << 8)));
            }
            P[i] = xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) P[i] ^= dpp<0x111, 0xF>(P[i]);  // row_shr:1
#pragma unroll
        for (int i = 0; i < NR; ++i) P[i] ^= dpp<0x112, 0xF>(P[i]);  // row_shr:2
#pragma unroll
        for (int i = 0; i < NR; ++i) P[i] ^= dpp<0x114, 0xF>(P[i]);  // row_shr:4
#pragma unroll
        for (int i = 0; i < NR; ++i) P[i] ^= dpp<0x118, 0xF>(P[i]);  // row_shr:8
#pragma unroll
        for (int i = 0; i < NR; ++i) P[i] ^= dpp<0x142, 0xA>(P[i]);  // row_bcast:15 -> rows 1, 3
#pragma unroll
        for (int i = 0; i < NR; ++i) P[i] ^= dpp<0x143, 0xC>(P[i]);  // row_bcast:31 -> rows 2, 3
#pragma unroll
        for (int i = 0; i < NR; ++i) pre[i] = dpp<0x138, 0xF>(P[i]);  // wave_shr:1 -> exclusive (lane 0: 0)
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const uint32_t j = j0 + i;
            // blocks of this slab holding a record end (the plan is zero past
            // the last row)
            const uint32_t m = (nib >> (4 * i)) & 15u;
            // the register at the start of block b (selects, no branches)
            auto cap = [&](uint32_t b) {
                uint32_t v = b == 3 ? c3[i] : c2[i];
                v = b == 1 ? c1[i] : v;
                return b == 0 ? 0u : v;
            };
            if (__ballot(m & (m - 1)) == 0) {
                // common case: at most one record end per slab, its slot is
                // the block's ends before this row + (cut lanes before)
                const uint64_t C = __ballot(m != 0);
                const uint32_t idx =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(C >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)C, 0u));
                store_ep(m ? (rel + idx) * 8u : kDrop, cap((uint32_t)__builtin_ctz(m | 16u)), pre[i]);
#ifdef GCK_XP_EBLK
                { const uint32_t bb = (uint32_t)__builtin_ctz(m | 16u) & 3u; store_blk(m ? (rel + idx) * 8u : kDrop, GCK_PICK_BLK(w[i], bb)); }
#endif
                rel += (uint32_t)__builtin_popcountll(C);
            } else {
                // a slab with 2..4 record ends (records under 64 B): ids by
                // an exclusive count over the lanes, four stores per lane
                const uint32_t n = __builtin_popcount(m);
                const uint32_t ex = wave_incl_sum(n) - n;
                uint32_t mm = m;
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    store_ep(q < n ? (rel + ex + q) * 8u : kDrop, cap((uint32_t)__builtin_ctz(mm | 16u)), pre[i]);
#ifdef GCK_XP_EBLK
                    { const uint32_t bb = (uint32_t)__builtin_ctz(mm | 16u) & 3u; store_blk(q < n ? (rel + ex + q) * 8u : kDrop, GCK_PICK_BLK(w[i], bb)); }
#endif
                    mm &= mm - 1;
                }
                rel += (uint32_t)__builtin_amdgcn_readlane((int)(ex + n), 63);
            }
            const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)P[i], 63);  // F(0, row)
            rend_buf = lane == j ? total : rend_buf;
        }
    };

    // prologue: this wave's first two blocks, the first plan
    GCK_CLK_BEGIN();
    uint64_t q = grab();
    if (q >= n_blocks) {
        GCK_CLK_END(0, w);
        return;
    }
    uint64_t qn = grab();
    Plan pc, pn;
    load_plan(q, pc);
    Batch bc, bn;
    load_plan(qn, pn);
    load_batch(pc, bc);
    // kPrefetch rows in flight per wavefront (row buffers rotate with period
    // NB, which divides the 4 steps of a quad, so every buffer has fixed
    // registers)
    static_assert(kPrefetch == 1 || (NR == 1 && kPrefetch <= 3), "prefetch depth > 1 needs one row per step");
    constexpr int NB = kPrefetch == 1 ? 2 : 4;
    RowBuf buf[NB][NR];
#pragma unroll
    for (int d = 0; d < kPrefetch; ++d) issue(q * kBlockRows + (uint64_t)d * NR, buf[d]);
    for (;;) {
        // block q: plan pc is resident; fetch the next block's plan and claim
        // the one after it (both land during this block)
        // pn (block qn) landed during the previous block: its record ends now,
        // the plan of the block after it next
        uint64_t qnn = 0;
        Plan pnn;
        load_batch(pn, bn);
        if constexpr (kLateQd < 0) {
            qnn = grab();
            load_plan(qnn, pnn);
        }
        const uint64_t row_b = q * kBlockRows;
        uint32_t rend_buf = 0;
        uint32_t rel = 0;  // record ends in the block's rows so far (at most one per 16 B block)
        ra0 = (uint32_t)__builtin_amdgcn_readlane((int)pc.ra, 0);  // the block's first record end
        ep_rsrc = make_rsrc(out_ep + ra0, 0x7FFFFFF0);
#ifdef GCK_XP_EBLK
        blk_rsrc = make_rsrc(out_blk + (uint64_t)ra0 * 16, 0x7FFFFFF0);
#endif
        uint32_t nibs[kNibDw];
        build_nibs(row_b, ra0, pc.re, &bc, nibs);
        // steps in quads: a quad of 4 steps consumes 4 NR plan nibbles per
        // lane; the two row buffers alternate, so each has fixed registers
        for (int qd = 0; qd < kSteps / 4; ++qd) {
            // this quad's nibbles (a uniform select: qd is a loop counter)
            uint32_t nib = nibs[0];
#pragma unroll
            for (int d = 1; d < kNibDw; ++d)
                if (qd * NR / 2 == d) nib = nibs[d];
            if constexpr (NR == 1) nib >>= 16 * (qd & 1);
            if constexpr (kLateQd >= 0) {
                if (qd == kLateQd) {  // (uniform)
                    qnn = grab();
                    load_plan(qnn, pnn);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int st = qd * 4 + u;
                // the rows kPrefetch steps ahead: this block, or the next block's first
                const int ahead = st + kPrefetch;
                const uint64_t nrow =
                    ahead < kSteps ? row_b + (uint64_t)ahead * NR : qn * kBlockRows + (uint64_t)(ahead - kSteps) * NR;
                issue(nrow, buf[(u + kPrefetch) % NB]);
                // keep the next row's loads here, ahead of this row's compute:
                // left alone, the scheduler sinks them past most of the chain
                // (reusing the current row's registers), so only one row was
                // in flight while the wave computed
                __builtin_amdgcn_sched_barrier(0);
                process(row_b + (uint64_t)st * NR, (uint32_t)(st * NR), nib >> (4 * NR * u), rel, buf[u % NB],
                        rend_buf);
            }
        }
        // the block's 64 rrow values, one coalesced store (rows past the end
        // to the scratch slots)
        *(lane < kBlockRows && row_b + lane < n_rows ? out_rend + row_b + lane : rend_scratch + lane) = rend_buf;
        if (qn >= n_blocks) {
            GCK_CLK_END(0, w);
            return;
        }
        q = qn;
        qn = qnn;
        pc = pn;
        pn = pnn;
        bc = bn;
    }
}


// ---------------------------------------------------------------- finalize ---
// Per record r = [rs, ve) (core/db.go:311 applied to every record).  Notation
// as in gck_math.h; for a position p inside row R (row end E_R):
//   A(p) = Z_{E_R - p}(F(0, [R*4096, p)))   the row's bytes before p, referenced to E_R.
// k_crc_rows gives, for the record end ve in block [bs, bs+16) of slab k:
//   c = F(0, [slab start, bs)),  pre = A(slab start),  so
//   A(ve) = pre ^ Z_{E - ve}(ft),  ft = F(c, [bs, ve))  (<= 16 bytes, here);
// and per row rrow = F(0, row).  Then, with fr / lr the rows of rs / ve - 1:
//   acc = A(ve) ^ A(rs)                                  (fr == lr)
//   acc = Horner_{Z_4096}(rrow[fr] ^ A(rs), rrow[fr+1..lr-1], A(ve))   (else)
//   F(0, [rs, ve)) = Z_{-(E - ve)}(acc) = ft ^ Z_{-(E - ve)}(acc ^ Z_{E-ve}(ft))
// (A(rs) = 0 when rs starts a row).  The header + key prefix is removed by
// linearity: F(0, value) = F(0, [rs, ve)) ^ Z_V(F(0, [rs, vs))), and
//   crc = F(0, value) ^ crc32(0^V).
// ft of record r-1 uses the 16 B block just before rs, which record r's lane
// reads next to its own header anyway: lane k computes it and hands it to
// lane k-1 (DPP); a lane whose successor is not its neighbour (wave end, file
// end, range end) reads its own end block.
// ValuePos = lastOffset + 16 + KeySize mod 2^32 (core/keydir.go:25), with
// lastOffset = carry + offset within the file.
// a * b mod P for a per-lane b and any a, by a 4-bit window over a:
// M[v] = b * (v3 + v2 x + v1 x^2 + v0 x^3) (v = a nibble, its bit 3 the lower
// power) in a wave-private LDS table, entry-major (entry v of lane l at
// byte mw + 256 v + 4 l: each lane of a 32-lane group on its own bank), then
// Horner from the highest-degree nibble with y * x^4 = (y >> 4) ^ R[y & 15].
// About 60 VALU + 15 LDS writes + 15 LDS reads, against ≈160 VALU for a
// branch-free bit-serial product (measured slower in any of finalize's four
// multiplies).
// M[0] must be zero (written once per kernel); mw = the wave's region + 4 lane;
// rb = the lane's copy of R (32 copies, entry e of copy l at + 128 e + 4 l:
// conflict-free, where one 16-entry copy put 32 lanes on 16 banks).
__device__ __forceinline__ uint32_t mulx(uint32_t v) {
    return (v >> 1) ^ (kPoly & (uint32_t)(-(int32_t)(v & 1u)));
}
__device__ __forceinline__ uint32_t gf_mul_lds(char *lds, uint32_t mw, uint32_t rb, uint32_t a, uint32_t b) {
    const uint32_t m8 = b, m4 = mulx(m8), m2 = mulx(m4), m1 = mulx(m2);
    const uint32_t m[16] = {0u, m1, m2, m1 ^ m2, m4, m4 ^ m1, m4 ^ m2, m4 ^ m2 ^ m1,
                            m8, m8 ^ m1, m8 ^ m2, m8 ^ m2 ^ m1, m8 ^ m4, m8 ^ m4 ^ m1, m8 ^ m4 ^ m2, m8 ^ m4 ^ m2 ^ m1};
#pragma unroll
    for (int v = 1; v < 16; ++v) *reinterpret_cast<uint32_t *>(lds + mw + 256 * v) = m[v];
    auto ent = [&](int t) {  // M[nibble t of a] (t = 7: bits 3..0, the highest powers)
        const int sh = 20 - 4 * t;
        const uint32_t x = sh >= 0 ? a >> sh : a << -sh;
        return *reinterpret_cast<const uint32_t *>(lds + ((x & 0xF00u) | mw));
    };
    uint32_t y = ent(7);
#pragma unroll
    for (int t = 6; t >= 0; --t) {
        const uint32_t r = *reinterpret_cast<const uint32_t *>(lds + (rb | ((y << 7) & 0x780u)));
        y = xor3(y >> 4, r, ent(t));
    }
    return y;
}
__device__ __forceinline__ uint32_t z4096(const uint32_t *Tz, uint32_t a) {
    return Tz[a & 0xFF] ^ Tz[256 + ((a >> 8) & 0xFF)] ^ Tz[512 + ((a >> 16) & 0xFF)] ^ Tz[768 + (a >> 24)];
}
// crc' = T3[b0] ^ T2[b1] ^ T1[b2] ^ T0[b3] for a = crc ^ word (T[k*256+b] = Tk[b])
__device__ __forceinline__ uint32_t slice4t(const uint32_t *T, uint32_t a) {
    return xor3(T[768 + (a & 0xFF)], T[512 + ((a >> 8) & 0xFF)], T[256 + ((a >> 16) & 0xFF)]) ^ T[a >> 24];
}
// F(c, the first nb (1..3) bytes of word y): (c >> 8nb) ^ slice4 of (c ^ y)
// moved up by 4 - nb bytes (the moved-out bytes index T[0] = 0).
__device__ __forceinline__ uint32_t partial_word(const uint32_t *T, uint32_t c, uint32_t y, uint32_t nb) {
    return (c >> (8 * nb)) ^ slice4t(T, (c ^ y) << (32 - 8 * nb));
}
// F(c, bytes [0, L)) of the 16 B block v, L in [0, 16].
__device__ __forceinline__ uint32_t crc_block(const uint32_t *T, uint32_t c, const uint4 &v, uint32_t L) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (4u * i + 4 <= L) c = slice4t(T, c ^ w[i]);
    const uint32_t nb = L & 3u, j = L >> 2;
    if (nb) c = partial_word(T, c, j == 0 ? w[0] : j == 1 ? w[1] : j == 2 ? w[2] : w[3], nb);
    return c;
}

// 8 wavefronts per workgroup share one set of tables, among them x^{-8d} for
// every d < 4096 (16 KiB: a lookup instead of a multiply; 61 KiB per
// workgroup, two per CU): 0.467-0.473 against 0.476-0.477 ms with 4
// wavefronts and the two-table multiply (profiles/r5k)
#ifndef GCK_FIN_XI
#define GCK_FIN_XI 1
#endif
#if GCK_FIN_XI
constexpr uint32_t kFinThreads = 512;
#else
constexpr uint32_t kFinThreads = 256;
#endif
constexpr uint32_t kFinWaves = kFinThreads / 64;
// HASH: also each record's key hash (kd_common.h key_hash, what k_kd_insert
// would compute) into khash[r], from the key words the record's header + key
// CRC already holds in registers, and the record into the keydir table ktab
// (kd_insert_rec, as k_kd_insert would: gck_ctx_keydir_hash)
template <bool HASH>
__global__ __launch_bounds__(kFinThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_finalize(const uint8_t *__restrict__ arena,
                                                  const uint64_t *__restrict__ rec_off,
                                                  const uint2 *__restrict__ rec_kv,
                                                  const uint32_t *__restrict__ rec_file,
                                                  const uint64_t *__restrict__ fbase,
                                                  const uint32_t *__restrict__ carry, const uint64_t *__restrict__ rng,
                                                  const uint2 *__restrict__ ep, const uint32_t *__restrict__ rend,
                                                  const uint32_t *__restrict__ g_slice,
                                                  const uint32_t *__restrict__ xinv,
                                                  const uint32_t *__restrict__ zrow,
                                                  const uint32_t *__restrict__ xa,
                                                  const uint32_t *__restrict__ xb, gck_rec *__restrict__ out,
                                                  uint32_t *counters, uint64_t *__restrict__ khash,
                                                  unsigned long long *__restrict__ ktab, uint64_t kmask,
                                                  uint32_t *__restrict__ kstat, uint32_t *mbox) {
    __shared__ uint32_t Tz[1024];  // Z_4096 as 4 byte tables
    __shared__ uint32_t T[1024];   // slicing-by-4 tables T0..T3
    // gf_mul_lds: one 4 KiB table region per wave, then R (y * x^4 = (y >> 4) ^
    // R[y & 15]) in 32 copies.  A wave's output staging (64 gck_rec = 2560 B)
    // reuses bytes 256.. of its region (the M entries 1..15, rewritten by every
    // gf_mul_lds; LDS operations of one wave execute in order)
    __shared__ uint32_t Gm[kFinWaves * 1024 + 512];
    // the shift constants every record needs, from small LDS tables instead
    // of random global loads (each a distinct line per lane for the TA):
    // x^{-8d}, d < 4096, as two 64-entry tables (d & 63, 64 (d >> 6)), and
    // x^{8v}, v < 65536, as two byte tables (v & 0xFF, 256 (v >> 8)); one
    // more multiply each
#if GCK_FIN_XI
    __shared__ uint32_t Xi[4096];  // x^{-8d}, d < 4096: no multiply
#else
    __shared__ uint32_t Xi[128];
#endif
    __shared__ uint32_t Xb[512];
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) {
        Tz[i] = zrow[i];
        T[i] = g_slice[i];
    }
#if GCK_FIN_XI
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) Xi[i] = xinv[i];
#else
    for (uint32_t i = threadIdx.x; i < 64; i += blockDim.x) {
        Xi[i] = xinv[i];
        Xi[64 + i] = xinv[64 * i];
    }
#endif
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
        Xb[i] = xb[i];
        Xb[256 + i] = xb[256 * i];
    }
    for (uint32_t i = threadIdx.x; i < 512; i += blockDim.x) Gm[kFinWaves * 1024 + i] = mulx(mulx(mulx(mulx(i >> 5))));
    Gm[(threadIdx.x >> 6) * 1024 + (threadIdx.x & 63)] = 0;  // entry 0 of every lane
    __shared__ uint32_t wg_next;  // the workgroup's next piece slot (its wavefronts claim from it)
    if (threadIdx.x == 0) wg_next = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    char *const ldsb = reinterpret_cast<char *>(Gm);  // byte offsets into Gm
    const uint32_t mw = (threadIdx.x >> 6) * 4096 + lane * 4, rxb = kFinWaves * 4096 + (lane & 31) * 4;
    uint4 *const Ost = reinterpret_cast<uint4 *>(ldsb + (threadIdx.x >> 6) * 4096 + 256);
    const uint64_t rb = rng[0], re = rng[1];
    uint32_t n_rej = 0;  // verdict rejects of this thread (summed per block at the end)
    // wave-uniform loop: the 64 lanes hold 64 consecutive records.  Loads in
    // three waves per iteration: the record table of this iteration (issued
    // one iteration ahead), then every load that depends on it at once (header
    // and key bytes, the end block where no neighbour provides ft, row sums,
    // shift tables), then the next iteration's record table, so the compute
    // below waits for one memory round trip per iteration.
    struct Rec {
        uint64_t rs;
        uint2 kv;       // (KeySize, ValueSize)
        uint32_t f;
        uint2 ep;       // (c, pre) of the record's end block
        uint32_t f0;    // rec_file / ep of the record before the wave's first
        uint2 ep0;
    };
    auto load_rec = [&](uint64_t base, Rec &o) {
        const uint64_t r = min(base + lane, re - 1), r0 = base ? base - 1 : 0;
        o.rs = rec_off[r];
        o.kv = rec_kv[r];
        o.f = rec_file[r];
        o.ep = ep[r];
        o.f0 = base ? rec_file[r0] : 0xFFFFFFFFu;
        o.ep0 = ep[r0];
    };
    // Per-iteration geometry of a wave's 64 records (recomputed where needed:
    // a few VALU, fewer registers than carrying it)
    struct Geo {
        bool valid, prev_same, have;
        uint32_t f, V, e_prev, pre_prev, d;
        uint64_t rs, vs, ve, bsp, bse, fr, lr, w0;
        uint2 kv;
    };
    auto geo = [&](const Rec &c, uint64_t b) {
        Geo g;
        g.valid = b + lane < re;
        g.rs = c.rs;
        g.kv = c.kv;
        g.f = c.f;
        g.V = c.kv.y;
        g.vs = g.rs + 16 + g.kv.x;
        g.ve = g.vs + g.V;
        // the previous record (r - 1): lane - 1's, or the wave's extra one
        const uint32_t f_prev = (uint32_t)__builtin_amdgcn_update_dpp((int)c.f0, (int)c.f, 0x138, 0xF, 0xF, false);
        g.e_prev = (uint32_t)__builtin_amdgcn_update_dpp((int)c.ep0.x, (int)c.ep.x, 0x138, 0xF, 0xF, false);
        g.pre_prev = (uint32_t)__builtin_amdgcn_update_dpp((int)c.ep0.y, (int)c.ep.y, 0x138, 0xF, 0xF, false);
        // records of a file are contiguous in walk order; lanes past the range
        // repeat the last record and have no predecessor
        g.prev_same = g.valid && f_prev == g.f;
        // ft of this record comes from lane + 1 if that lane holds record r + 1 of the same file
        const uint64_t nb_same = __ballot(g.valid && g.prev_same);
        g.have = lane < 63 && ((nb_same >> (lane + 1)) & 1);
        g.bsp = g.prev_same ? (g.rs - 1) & ~15ull : g.rs;
        g.bse = (g.ve - 1) & ~15ull;
        g.fr = g.rs / kRow;
        g.lr = (g.ve - 1) / kRow;
        g.d = (uint32_t)((g.lr + 1) * kRow - g.ve);
        g.w0 = g.rs & ~3ull;
        return g;
    };
    // every load that depends on the record table
    struct Dep {
        uint4 vp, vend;
        uint32_t pw[12], rr[12];
        uint32_t xhi, cf;
        uint64_t fb;
#ifdef GCK_FIN_GTAB
        uint32_t xi, xv;
#endif
    };
    auto issue = [&](const Geo &g, Dep &o) {
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(arena + g.w0);
        // block holding byte rs - 1: only a record with a predecessor in its
        // file needs it (ft_prev; without one, bsp = rs and it is unused)
        o.vp = make_uint4(0, 0, 0, 0);
        if (g.prev_same) o.vp = *reinterpret_cast<const uint4 *>(arena + g.bsp);
        // header + keys up to 24 B as three 16 B loads (dword aligned; the
        // arena is padded): every load instruction of a wave touches 64
        // records' lines, so the count of instructions, not bytes, is the cost
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            // (the third only when the prefix [w0, vs) reaches its words:
            // keys under 12 + (4 - lead) bytes end in the first 32)
            u32x4_a4 v = {0u, 0u, 0u, 0u};
            if (i < 2 || g.vs - g.w0 >= 32) v = reinterpret_cast<const u32x4_a4 *>(wp)[i];
            o.pw[4 * i] = v.x;
            o.pw[4 * i + 1] = v.y;
            o.pw[4 * i + 2] = v.z;
            o.pw[4 * i + 3] = v.w;
        }
        o.vend = make_uint4(0, 0, 0, 0);
        if (!g.have)
            o.vend = *reinterpret_cast<const uint4 *>(arena + g.bse);
        // row sums rend[fr .. fr + 11] the record crosses (up to three 16 B
        // loads, rend is padded; only the ones a record spanning rows uses:
        // most records lie inside one row)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            u32x4_a4 v = {0u, 0u, 0u, 0u};
            if (g.lr > g.fr + 4 * i) v = reinterpret_cast<const u32x4_a4 *>(rend + g.fr)[i];
            o.rr[4 * i] = v.x;
            o.rr[4 * i + 1] = v.y;
            o.rr[4 * i + 2] = v.z;
            o.rr[4 * i + 3] = v.w;
        }
        o.xhi = g.V >= 65536 ? xa[g.V >> 16] : 0u;
#ifdef GCK_FIN_GTAB
        o.xi = xinv[g.d];          // x^{-8d}, d < 4096 (16 KiB table, L2)
        o.xv = xb[g.V & 0xFFFFu];  // x^{8 (V mod 2^16)} (256 KiB table, L2)
#endif
        o.cf = carry[g.f];
        o.fb = fbase[g.f];
    };
    auto compute = [&](const Rec &c, const Geo &g, const Dep &o, uint64_t base) {
        const bool valid = g.valid, prev_same = g.prev_same, have = g.have;
        const uint64_t rs = g.rs, vs = g.vs, ve = g.ve, bsp = g.bsp, bse = g.bse, fr = g.fr, lr = g.lr, w0 = g.w0;
        const uint2 kv = g.kv;
        const uint32_t f = g.f, V = g.V, e_prev = g.e_prev, pre_prev = g.pre_prev;
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(arena + w0);
        const uint4 vp = o.vp, vend = o.vend;
        const uint32_t *pw = o.pw, *rr = o.rr;
        const uint32_t xhi = o.xhi, cf = o.cf;
        const uint64_t fb = o.fb;
        // ---- compute
        const uint32_t ft_prev = crc_block(T, e_prev, vp, (uint32_t)(rs - bsp));
        // A(rs) = pre_prev ^ Z_{E-rs}(ft_prev) (0 when rs starts a row).  Only
        // pre_prev enters the row sums: they then give F(s, [rs, ve)) with
        // s = ft_prev, and the header + key CRC below starts from s too, so
        // F(0, value) = F(s, [rs, ve)) ^ Z_V(F(s, [rs, vs))) needs no shift of s.
        const bool mid = prev_same && (rs & (kRow - 1)) != 0;
        const uint32_t a_rs = mid ? pre_prev : 0u, s0 = mid ? ft_prev : 0u;
        const uint32_t ft_next = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ft_prev, 0x130, 0xF, 0xF, false);  // wave_shl:1
        const uint32_t ft = have ? ft_next : crc_block(T, c.ep.x, vend, (uint32_t)(ve - bse));
        // acc = the record's bytes of its rows, referenced to the end row's
        // end, without the last block's ft (added back unshifted below)
        uint32_t acc = c.ep.y;
        if (fr == lr) {
            acc ^= a_rs;
        } else {
            uint32_t h_acc = rr[0] ^ a_rs;
#pragma unroll
            for (int j = 1; j < 12; ++j)
                if (fr + j < lr) h_acc = z4096(Tz, h_acc) ^ rr[j];
            for (uint64_t row = fr + 12; row < lr; ++row) h_acc = z4096(Tz, h_acc) ^ rend[row];  // records over 48 KiB
            acc ^= z4096(Tz, h_acc);
        }
        // F(s, [rs, ve)) = ft ^ Z_{-(E-ve)}(acc)
        // (a bit-serial VALU product in place of any of these four measured
        // slower: 0.47-0.64 ms against 0.46-0.47, profiles/r3j/ab_finvalu.log)
        auto mul = [&](uint32_t a, uint32_t b) { return gf_mul_lds(ldsb, mw, rxb, a, b); };
#if defined(GCK_FIN_GTAB)
        const uint32_t xi = o.xi;
#elif GCK_FIN_XI
        const uint32_t xi = Xi[g.d];  // x^{-8d}
#else
        const uint32_t xi = mul(Xi[64 + (g.d >> 6)], Xi[g.d & 63]);  // x^{-8d}
#endif
        const uint32_t chain = ft ^ mul(xi, acc);
        // F(s, prefix): header + key bytes [rs, vs) as aligned words from
        // rs & ~3; the first word's bytes before rs are shifted out
        // (partial_word over its last 4 - lead bytes)
        const uint32_t lead = (uint32_t)(rs & 3), L = (uint32_t)(vs - w0);
        const uint32_t hcrc = ab(pw[1], pw[0], lead), hts = ab(pw[2], pw[1], lead);  // header CRC, Timestamp
        // word 0: F(s0, its bytes lead..3) = (s0 >> 8nb) ^ slice4((s0 ^ w >> 8 lead) << 8 lead), nb = 4 - lead
        uint32_t p = slice4t(T, (s0 ^ (pw[0] >> (8 * lead))) << (8 * lead)) ^ (lead ? s0 >> (32 - 8 * lead) : 0u);
        // unrolled over the words in registers (no indexed register array),
        // then the words of long keys from memory
        const uint32_t nw = L / 4;
        uint32_t y = 0;
#pragma unroll
        for (uint32_t i = 1; i < 12; ++i) {
            if (i < nw) p = slice4t(T, p ^ pw[i]);
            y = i == nw ? pw[i] : y;
        }
        for (uint32_t i = 12; i < nw; ++i) p = slice4t(T, p ^ wp[i]);
        if (nw >= 12) y = wp[nw];
        if (L & 3) p = partial_word(T, p, y, L & 3);  // L >= 16: y is never the masked word
        // x^(8V) = xa[V >> 16] * x^(8 (V & 0xFF00)) * x^(8 (V & 0xFF))
#ifdef GCK_FIN_GTAB
        uint32_t xv = o.xv;
#else
        uint32_t xv = mul(Xb[256 + ((V >> 8) & 0xFF)], Xb[V & 0xFF]);
#endif
        if (V >= 65536) xv = mul(xhi, xv);
        // crc = F(0, value) ^ crc32(0^V), crc32(0^V) = Z_V(~0) ^ ~0, and Z_V is
        // linear: one multiply covers the prefix and the init term (no
        // crc32(0^V) table load)
        const uint32_t calc = chain ^ mul(xv, p ^ 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
        {
            // The wave's records are consecutive gck_recs (40 B each): staged in
            // LDS, then stored as 16 B per lane, 1 KiB contiguous per instruction
            // (three 8/16 B stores per lane at a 40 B stride write partial lines)
            const uint64_t fo = rs - fb;
            const bool tomb = kv.x == 0;
            uint2 *sl = reinterpret_cast<uint2 *>(reinterpret_cast<char *>(Ost) + lane * sizeof(gck_rec));
            sl[0] = make_uint2((uint32_t)fo, (uint32_t)(fo >> 32));                    // rec_off
            sl[1] = make_uint2(f, tomb ? kv.y : kv.x);                                 // file, key_len
            sl[2] = make_uint2(cf + (uint32_t)fo + 16u + kv.x, kv.y);                  // value_pos, value_size
            sl[3] = make_uint2(hcrc, hts);                                             // crc, ts
            sl[4] = make_uint2((tomb ? GCK_F_TOMBSTONE : 0u) | (calc == hcrc ? GCK_F_CRC_OK : 0u), calc);
            __builtin_amdgcn_wave_barrier();
            const uint32_t nbytes = (uint32_t)min(re - base, (uint64_t)64) * (uint32_t)sizeof(gck_rec);
            char *dst = reinterpret_cast<char *>(out + base);
#pragma unroll
            for (uint32_t k = 0; k < 3; ++k) {
                const uint32_t off = k * 1024 + lane * 16;
                const uint4 v = Ost[off / 16];
                if (off + 16 <= nbytes) {
                    *reinterpret_cast<u32x4_a4 *>(dst + off) = u32x4_a4{v.x, v.y, v.z, v.w};
                } else if (off < nbytes) {  // an odd record count ends mid-chunk
                    *reinterpret_cast<uint2 *>(dst + off) = make_uint2(v.x, v.y);
                }
            }
            __builtin_amdgcn_wave_barrier();
            n_rej += valid && calc != hcrc;
            if constexpr (HASH) {
                // key_hash (kd_common.h) of the record's key: KeySize bytes at
                // rs + 16, or ValueSize for a tombstone (core/db.go:151-155).
                // A Put's key of up to 28 - lead bytes is in pw (words 4..11,
                // byte shift lead); other keys are read again.
                const uint32_t klen = kv.x ? kv.x : kv.y;
                uint64_t hh = 0x9E3779B97F4A7C15ull ^ ((uint64_t)klen << 32);
                if (kv.x != 0 && klen + lead <= 28) {
#pragma unroll
                    for (uint32_t i = 0; i < 7; ++i) {
                        if (4 * i < klen) {
                            uint32_t v = __builtin_amdgcn_alignbyte(pw[5 + i], pw[4 + i], lead);
                            const uint32_t left = klen - 4 * i;
                            v = left >= 4 ? v : v & ((1u << (8 * left)) - 1u);
                            hh = mix64d(hh ^ v) + i;
                        }
                    }
                } else {
                    const KeyWords k(arena, rs + 16, klen);
                    for (uint32_t i = 0; 4 * i < klen; ++i) hh = mix64d(hh ^ k[i]) + i;
                }
                if (valid && ktab) {  // (no table: a run too large for one; gck_ctx_keydir refuses it)
                    const uint64_t h = mix64d(hh);
                    khash[base + lane] = h;
                    bool ok;
                    if (kv.x != 0 && klen + lead <= 28) {
                        // the key words as values (an indexed register array
                        // would go to scratch)
                        const uint32_t k0 = ab(pw[5], pw[4], lead), k1 = ab(pw[6], pw[5], lead),
                                       k2 = ab(pw[7], pw[6], lead), k3 = ab(pw[8], pw[7], lead),
                                       k4 = ab(pw[9], pw[8], lead), k5 = ab(pw[10], pw[9], lead),
                                       k6 = ab(pw[11], pw[10], lead);
                        ok = kd_insert_rec(arena, rec_off, rec_kv, ktab, kmask, h, base + lane, kv.x == 0,
                                      [=](uint32_t i) {
                                          const uint32_t v = i == 0   ? k0
                                                             : i == 1 ? k1
                                                             : i == 2 ? k2
                                                             : i == 3 ? k3
                                                             : i == 4 ? k4
                                                             : i == 5 ? k5
                                                                      : k6;
                                          const uint32_t left = klen - 4 * i;
                                          return left >= 4 ? v : v & ((1u << (8 * left)) - 1u);
                                      },
                                      klen);
                    } else {
                        const KeyWords k(arena, rs + 16, klen);
                        ok = kd_insert_rec(arena, rec_off, rec_kv, ktab, kmask, h, base + lane, kv.x == 0, [&](uint32_t i) { return k[i]; }, klen);
                    }
                    if (!ok) atomicOr(kstat, 1u);  // gck_ctx_keydir builds the table again
                }
            }
        }
    };
    // The record table one iteration ahead, the loads that depend on it
    // issued together and waited for, then the compute.  (Loading the table
    // two iterations ahead and the dependent loads one ahead measured slower:
    // 0.517-0.520 vs 0.496-0.498 ms)
    GCK_CLK_BEGIN();
#ifdef GCK_CLOCK_STAMPS
    // stamps build only: per wavefront, the shader cycles spent waiting for
    // an iteration's loads (forced vmcnt(0)) and computing it
    uint64_t fin_wait = 0, fin_comp = 0;
#endif
    // 64-record pieces.  Workgroup b owns pieces b, b + NB, b + 2 NB, ... (NB
    // workgroups: every workgroup samples the whole corpus) and its wavefronts
    // take them one at a time from an LDS counter, each claim issued an
    // iteration before its piece is loaded.  A wavefront's fixed stride of 39
    // C3 pieces took 354-443 us (p10-max, profiles/r6c: pieces of long records
    // cost more); sharing a workgroup's 312 pieces among its 8 wavefronts
    // evens that out.  (A global queue for the last quarter of the pieces made
    // the kernel 0.79 ms: 40 K claims on one address serialise, profiles/r6d.)
    // From the last piece back when the keys are inserted here (a key's later
    // record then mostly claims its slot first, as in k_kd_insert).
    const uint64_t npc = re > rb ? (re - rb + 63) / 64 : 0, NB = gridDim.x;
    auto at = [&](uint64_t k) { return rb + 64 * (HASH ? npc - 1 - k : k); };
    auto claim = [&]() {  // lane 0: the wavefront's next slot of its workgroup's pieces
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(&wg_next, 1u);
        return v;
    };
    auto piece = [&](uint32_t v) { return blockIdx.x + NB * (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
    uint64_t pc = piece(claim());
    uint32_t vn = claim();  // the piece after pc (read at the end of the first iteration)
    Rec cur, nxt;
    if (pc < npc) load_rec(at(pc), cur);
    uint64_t pn = piece(vn);
    while (pc < npc) {
        const uint64_t base = at(pc);
        const Geo g = geo(cur, base);
        Dep dc;
        issue(g, dc);
        if (pn < npc) load_rec(at(pn), nxt);
        vn = claim();  // the piece after pn, in flight during this compute
#ifdef GCK_CLOCK_STAMPS
        const uint64_t fa = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t fb = __builtin_amdgcn_s_memtime();
        fin_wait += fb - fa;
#endif
        compute(cur, g, dc, base);
#ifdef GCK_CLOCK_STAMPS
        fin_comp += __builtin_amdgcn_s_memtime() - fb;
#endif
        cur = nxt;
        pc = pn;
        pn = piece(vn);
    }
#ifdef GCK_CLOCK_STAMPS
    if ((threadIdx.x & 63) == 0 && blockIdx.x * kFinWaves + (threadIdx.x >> 6) < kClkWaves) {
        g_fin_split[2 * (blockIdx.x * kFinWaves + (threadIdx.x >> 6))] = fin_wait;
        g_fin_split[2 * (blockIdx.x * kFinWaves + (threadIdx.x >> 6)) + 1] = fin_comp;
    }
#endif
    GCK_CLK_END(5, blockIdx.x * kFinWaves + (threadIdx.x >> 6));
    // one global atomic per block (per-record or per-wavefront atomics on one
    // address serialise: C5 has ~100k rejects)
    __shared__ uint32_t blk_rej;
    if (threadIdx.x == 0) blk_rej = 0;
    __syncthreads();
    const uint32_t wsum = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(n_rej), 63);
    if ((threadIdx.x & 63) == 0 && wsum) atomicAdd(&blk_rej, wsum);
    __syncthreads();
    if (!mbox) {
        if (threadIdx.x == 0 && blk_rej) atomicAdd(&counters[CNT_REJECT], blk_rej);
        return;
    }
    // device path: one 64-bit atomic per workgroup carries its rejects (low
    // 40 bits) and its arrival (bit 40 up); the workgroup that arrives last
    // knows the total and publishes the run's 32 counters / results into the
    // mapped host mailbox (the others were written by earlier kernels).  A
    // k_publish launch after finalize cost ~4 us and a dispatch per step; a
    // fence per workgroup before a separate ticket cost about as much.
    __shared__ uint64_t prior;
    if (threadIdx.x == 0)
        prior = atomicAdd(reinterpret_cast<unsigned long long *>(counters + CNT_FINTICKET),
                          (1ull << 40) + blk_rej);
    __syncthreads();
    if ((prior >> 40) == gridDim.x - 1 && threadIdx.x < 32) {
        uint32_t v = counters[threadIdx.x];
        if (threadIdx.x == CNT_REJECT) v = (uint32_t)((prior & ((1ull << 40) - 1)) + blk_rej);
        __hip_atomic_store(mbox + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ------------------------------------------------------------- host side ---
static void make_tables(std::vector<uint32_t> &slice, std::vector<uint32_t> &nib, std::vector<uint32_t> &xinv,
                        std::vector<uint32_t> &xa, std::vector<uint32_t> &xb, std::vector<uint32_t> &zrow) {
    slice.assign(4 * 256, 0);
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
        slice[n] = c;
    }
    for (int t = 1; t < 4; ++t)
        for (uint32_t n = 0; n < 256; ++n)
            slice[t * 256 + n] = (slice[(t - 1) * 256 + n] >> 8) ^ slice[slice[(t - 1) * 256 + n] & 0xff];
    // the wave CRC's lane shifts and Z_512 after the slicing tables
    // (gck_crc_wave.h: kGLs, kGZ512)
    slice.resize(kGTabWords, 0);
    for (uint32_t l = 0; l < 32; ++l) {
        const uint32_t K = xpow8n(16ull * (31 - l));
        for (uint32_t q = 0; q < 8; ++q)
            for (uint32_t v = 0; v < 16; ++v) slice[kGLs + q * 512 + v * 32 + l] = multmodp(K, v << (4 * q));
    }
    const uint32_t z5 = xpow8n(512);
    for (int k = 0; k < 4; ++k)
        for (uint32_t b = 0; b < 256; ++b) slice[kGZ512 + k * 256 + b] = multmodp(z5, b << (8 * k));
    nib.assign(64 * 8 * 16, 0);
    for (int l = 0; l < 64; ++l) {
        const uint32_t K = xpow8n((uint64_t)kSlab * (63 - l));
        for (int q = 0; q < 8; ++q)
            for (uint32_t v = 1; v < 16; ++v) nib[(l * 8 + q) * 16 + v] = multmodp(K, v << (4 * q));
    }
    uint32_t xinv8 = kX0;
    for (int i = 0; i < 8; ++i) xinv8 = multmodp(xinv8, kXinv);
    xinv.assign(kRow, 0);
    xinv[0] = kX0;
    for (int d = 1; d < kRow; ++d) xinv[d] = multmodp(xinv[d - 1], xinv8);
    xa.assign(65536, 0);
    xb.assign(65536, 0);
    xa[0] = xb[0] = kX0;
    const uint32_t s16 = xpow8n(65536), s1 = kX0 >> 8;
    for (int i = 1; i < 65536; ++i) {
        xa[i] = multmodp(xa[i - 1], s16);
        xb[i] = multmodp(xb[i - 1], s1);
    }
    const uint32_t x_row = xpow8n(kRow);
    zrow.assign(1024, 0);
    for (int k = 0; k < 4; ++k)
        for (uint32_t b = 1; b < 256; ++b) zrow[k * 256 + b] = multmodp(x_row, b << (8 * k));
}

static int ctx_init(Ctx *c, const gck_opts *o) {
    gck_opts d{};
    d.device = 0;
    d.chunk_bytes = 512 << 10;
    d.max_key = 65536;
    d.chunk_cap = 1024;
    d.spec_window = 0;  // the whole chunk
    if (o) {
        d.device = o->device;
        if (o->chunk_bytes) d.chunk_bytes = o->chunk_bytes;
        if (o->max_key) d.max_key = o->max_key;
        if (o->chunk_cap) d.chunk_cap = o->chunk_cap;
        if (o->spec_window) d.spec_window = o->spec_window;
        d.flags = o->flags;
    }
    if (d.chunk_bytes < 4096 || (d.chunk_bytes & (d.chunk_bytes - 1))) return GCK_EINVAL;
    if (d.spec_window == 0 || d.spec_window > d.chunk_bytes) d.spec_window = d.chunk_bytes;
    d.spec_window = (d.spec_window + 4095u) & ~4095u;  // whole 4 KiB search windows
    c->opts = d;
    c->chunk_shift = (uint32_t)__builtin_ctz(d.chunk_bytes);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= d.device || d.device < 0) {
        set_error("hipGetDeviceCount", hipErrorNoDevice, __FILE__, __LINE__);
        return GCK_EDEVICE;
    }
    GCK_HIP(hipSetDevice(d.device));
    hipDeviceProp_t prop;
    GCK_HIP(hipGetDeviceProperties(&prop, d.device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error("device is not gfx950", hipErrorInvalidDevice, __FILE__, __LINE__);
        return GCK_EDEVICE;
    }
    c->device = d.device;
    c->n_cu = prop.multiProcessorCount;
    int bpc = 0, bph = 0;
    GCK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, reinterpret_cast<const void *>(k_finalize<false>), kFinThreads, 0));
    GCK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bph, reinterpret_cast<const void *>(k_finalize<true>), kFinThreads, 0));
    c->fin_blocks_per_cu = bpc > 0 ? bpc : 1;
    c->fin_blocks_per_cu_hash = bph > 0 ? bph : 1;
    GCK_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (auto &e : c->ev) GCK_HIP(hipEventCreate(&e));
    if (multmodp(kXinv, kX0 >> 1) != kX0) return GCK_EINVAL;
    // the constant tables are the same for every context: built once per process
    struct Tables {
        std::vector<uint32_t> slice, nib, xinv, xa, xb, zrow;
        Tables() { make_tables(slice, nib, xinv, xa, xb, zrow); }
    };
    static const Tables tabs;
    const std::vector<uint32_t> &slice = tabs.slice, &nib = tabs.nib, &xinv = tabs.xinv,
                                &xa = tabs.xa, &xb = tabs.xb, &zrow = tabs.zrow;
    int rc;
    if ((rc = c->d_slice.ensure(slice.size() * 4)) || (rc = c->d_nib.ensure(nib.size() * 4)) ||
        (rc = c->d_xinv.ensure(xinv.size() * 4)) || (rc = c->d_xa.ensure(xa.size() * 4)) ||
        (rc = c->d_xb.ensure(xb.size() * 4)) || (rc = c->d_zrow.ensure(zrow.size() * 4)) ||
        (rc = c->d_counters.ensure(128)))
        return rc;
    {
        void *hp = nullptr, *dp = nullptr;
        GCK_HIP(hipHostMalloc(&hp, 128, hipHostMallocMapped | hipHostMallocCoherent));
        c->h_mbox = static_cast<uint32_t *>(hp);
        GCK_HIP(hipHostGetDevicePointer(&dp, hp, 0));
        c->d_mbox = static_cast<uint32_t *>(dp);
    }
    GCK_HIP(hipMemcpy(c->d_zrow.p, zrow.data(), zrow.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_slice.p, slice.data(), slice.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_nib.p, nib.data(), nib.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_xinv.p, xinv.data(), xinv.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_xa.p, xa.data(), xa.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_xb.p, xb.data(), xb.size() * 4, hipMemcpyHostToDevice));
    return GCK_OK;
}

static void ctx_free(Ctx *c) {
    DBuf *all[] = {&c->arena, &c->d_fbase, &c->d_flen, &c->d_ffirst, &c->d_fnch, &c->d_fbad, &c->d_fterm,
                   &c->d_ftpos, &c->d_fnrec, &c->d_ffirstrec, &c->d_carry, &c->d_ch_file, &c->d_ch_start,
                   &c->d_ch_end, &c->d_ch_wend, &c->d_ch_aentry, &c->d_ch_entry, &c->d_ch_exit, &c->d_ch_count, &c->d_ch_term, &c->d_ch_tpos, &c->d_ch_bad,
                   &c->d_rec_base, &c->d_bsum, &c->d_stage, &c->d_counters, &c->d_rec_off,
                   &c->d_rec_kv, &c->d_rec_file, &c->d_ep, &c->d_out, &c->d_blk_first, &c->d_rend,
                   &c->d_slice, &c->d_nib, &c->d_xinv, &c->d_xa, &c->d_xb, &c->d_zrow,
                   &c->d_freset, &c->d_gbase, &c->d_queue, &c->d_khash, &c->d_ktab, &c->d_kdstat, &c->d_live, &c->d_ktile,
                   &c->d_kdout, &c->d_kdidx, &c->d_kpart, &c->d_kcrank, &c->d_kbrank, &c->d_kpsum, &c->d_kptot,
                   &c->d_mkoff, &c->d_mtab, &c->d_mlive, &c->d_msrc, &c->d_mhdr, &c->d_mkeys, &c->d_mout,
                   &c->d_gkeys, &c->d_gkoff, &c->d_gstat, &c->d_gitem, &c->d_gvsize, &c->d_gexp, &c->d_gcrc,
                   &c->d_gvoff, &c->d_gvals, &c->d_gscan, &c->d_cpos, &c->d_chpos, &c->d_cbsum, &c->d_cfstart, &c->d_cnf,
                   &c->d_cdata, &c->d_chint, &c->d_cfoot, &c->d_cjmp, &c->d_con, &c->d_klb, &c->d_koff, &c->d_keyblob};
    for (DBuf *b : all) b->release();
    if (c->h_mbox) (void)hipHostFree(c->h_mbox);
    c->h_mbox = c->d_mbox = nullptr;
    if (c->h_up) (void)hipHostFree(c->h_up);
    c->h_up = c->d_up = nullptr;
    c->up_cap = 0;
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    c->stream = nullptr;
}

// Layout tables from pinned, mapped host memory (Ctx::h_up) into device
// buffers: up to 8 segments of 4-byte words, one grid dimension each.
struct UpSeg {
    uint32_t *dst;
    uint64_t src_off, words;
};
struct UpList {
    UpSeg seg[8];
};
__global__ void k_upload(const uint8_t *__restrict__ src, UpList l) {
    const UpSeg sg = l.seg[blockIdx.y];
    const uint32_t *s = reinterpret_cast<const uint32_t *>(src + sg.src_off);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < sg.words; i += (uint64_t)gridDim.x * blockDim.x)
        sg.dst[i] = s[i];
}

// Place files (walk order) in the arena and build the chunk table.
int ctx_layout(Ctx *c, const uint64_t *lens, uint32_t nfiles, const uint8_t *reset_after) {
    GCK_HIP(hipSetDevice(c->device));
    c->nfiles = nfiles;
    // new files: the last keydir's key count says nothing about them (a
    // pooled ring context may have held another group or database); the next
    // table is sized from the run's own record count
    c->kd_keys_hint = 0;
    c->f_base.assign(nfiles, 0);
    c->f_len.assign(lens, lens + nfiles);
    c->f_reset.assign(reset_after, reset_after + nfiles);
    c->f_first_chunk.assign(nfiles, 0);
    c->f_nchunks.assign(nfiles, 0);
    uint64_t pos = 0, data = 0;
    const uint64_t CB = c->opts.chunk_bytes;
    std::vector<uint32_t> ch_file;
    std::vector<uint64_t> ch_start, ch_end;
    for (uint32_t f = 0; f < nfiles; ++f) {
        c->f_base[f] = pos;
        pos += (lens[f] + kRow - 1) / kRow * kRow;
        data += lens[f];
        c->f_first_chunk[f] = (uint32_t)ch_file.size();
        for (uint64_t s = 0; s < lens[f]; s += CB) {
            ch_file.push_back(f);
            ch_start.push_back(s);
            ch_end.push_back(s + CB < lens[f] ? s + CB : lens[f]);
        }
        c->f_nchunks[f] = (uint32_t)ch_file.size() - c->f_first_chunk[f];
    }
    if (ch_file.size() >= 0xFFFFFFF0ull) return GCK_EINVAL;
    c->arena_len = pos;
    c->data_bytes = data;
    c->n_rows = pos / kRow;
    c->n_chunks = (uint32_t)ch_file.size();
    const uint64_t nc = c->n_chunks, nf = nfiles ? nfiles : 1;
    const uint64_t cap = c->opts.chunk_cap;
    int rc;
    // slack past the last file: k_spec_entry reads up to three 4 KiB windows
    // (+80 B) beyond a chunk end
    const bool fresh = c->arena.cap < pos + 5 * kRow;
    if ((rc = c->arena.ensure(pos + 5 * kRow))) return rc;
    if (fresh) GCK_HIP(hipMemset(c->arena.p, 0, c->arena.cap));
    if ((rc = c->d_fbase.ensure(nf * 8)) || (rc = c->d_flen.ensure(nf * 8)) || (rc = c->d_ffirst.ensure(nf * 4)) ||
        (rc = c->d_fnch.ensure(nf * 4)) || (rc = c->d_fbad.ensure(nf * 4)) || (rc = c->d_fterm.ensure(nf * 4)) ||
        (rc = c->d_ftpos.ensure(nf * 8)) || (rc = c->d_fnrec.ensure(nf * 8)) ||
        (rc = c->d_ffirstrec.ensure(nf * 8)) || (rc = c->d_carry.ensure(nf * 4)) ||
        (rc = c->d_ch_file.ensure((nc + 1) * 4)) || (rc = c->d_ch_start.ensure((nc + 1) * 8)) ||
        (rc = c->d_ch_end.ensure((nc + 1) * 8)) || (rc = c->d_ch_entry.ensure((nc + 1) * 8)) ||
        (rc = c->d_ch_wend.ensure((nc + 1) * 8)) || (rc = c->d_ch_aentry.ensure((nc + 1) * 8)) ||
        (rc = c->d_ch_exit.ensure((nc + 1) * 8)) || (rc = c->d_ch_count.ensure((nc + 1) * 4)) ||
        (rc = c->d_ch_term.ensure((nc + 1) * 4)) || (rc = c->d_ch_tpos.ensure((nc + 1) * 8)) || (rc = c->d_ch_bad.ensure((nc + 1) * 4)) ||
        (rc = c->d_rec_base.ensure((nc + 1) * 8)) || (rc = c->d_bsum.ensure((nc / kScanBlock + 4) * 8)) || (rc = c->d_freset.ensure(nf * 4)) ||
        (rc = c->d_gbase.ensure(kGbWords * 8)) || (rc = c->d_stage.ensure((nc + kStageIl) / kStageIl * kStageIl * (cap + 1) * 8)) || (rc = c->d_blk_first.ensure(((c->n_rows + kBlockRows - 1) / kBlockRows + 1) * 4)) ||
        (rc = c->d_rend.ensure((c->n_rows + 64) * 4)) ||
        (rc = c->d_queue.ensure(kQueueSlots * 4)))
        return rc;
    // k_scan_chunks' look-back words and tickets start zeroed (each launch
    // leaves them so)
    GCK_HIP(hipMemsetAsync(c->d_bsum.p, 0, c->d_bsum.cap, c->stream));
    // the tables, staged in pinned mapped host memory and copied by k_upload
    // on the context's stream (the previous upload has been consumed: the
    // stream is drained first, and runs are synchronous)
    std::vector<uint32_t> rs(reset_after, reset_after + nfiles);
    struct {
        void *dst;
        const void *src;
        uint64_t bytes;
    } tab[8] = {{c->d_fbase.p, c->f_base.data(), nfiles * 8ull},     {c->d_flen.p, c->f_len.data(), nfiles * 8ull},
                {c->d_ffirst.p, c->f_first_chunk.data(), nfiles * 4ull}, {c->d_fnch.p, c->f_nchunks.data(), nfiles * 4ull},
                {c->d_freset.p, rs.data(), nfiles * 4ull},              {c->d_ch_file.p, ch_file.data(), nc * 4},
                {c->d_ch_start.p, ch_start.data(), nc * 8},             {c->d_ch_end.p, ch_end.data(), nc * 8}};
    uint64_t up = 0;
    for (auto &t : tab) up += (t.bytes + 15) & ~15ull;
    GCK_HIP(hipStreamSynchronize(c->stream));
    if (up > c->up_cap) {
        if (c->h_up) (void)hipHostFree(c->h_up);
        c->h_up = c->d_up = nullptr;
        c->up_cap = 0;
        void *hp = nullptr, *dp = nullptr;
        if (hipHostMalloc(&hp, up, hipHostMallocMapped) != hipSuccess) return GCK_ENOMEM;
        c->h_up = static_cast<uint8_t *>(hp);
        GCK_HIP(hipHostGetDevicePointer(&dp, hp, 0));
        c->d_up = static_cast<uint8_t *>(dp);
        c->up_cap = up;
    }
    UpList l{};
    uint64_t off = 0, most = 0;
    for (int k = 0; k < 8; ++k) {
        if (tab[k].bytes) memcpy(c->h_up + off, tab[k].src, tab[k].bytes);
        l.seg[k] = UpSeg{static_cast<uint32_t *>(tab[k].dst), off, tab[k].bytes / 4};
        most = std::max<uint64_t>(most, tab[k].bytes / 4);
        off += (tab[k].bytes + 15) & ~15ull;
    }
    if (most) {
        const uint32_t gx = (uint32_t)std::min<uint64_t>((most + 255) / 256, 1024);
        k_upload<<<dim3(gx, 8), 256, 0, c->stream>>>(c->d_up, l);
        GCK_HIP(hipGetLastError());
    }
    return GCK_OK;
}

static inline uint32_t nblk(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }


static void launch_fixup(Ctx *c, hipStream_t s, uint32_t c0, uint32_t c1, const uint32_t *bad_cnt = nullptr) {
    k_fixup<<<nblk(c1 - c0, 256), 256, 0, s>>>(
        c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(), c->d_ch_file.as<uint32_t>(),
        c->d_ch_end.as<uint64_t>(), c->d_ffirst.as<uint32_t>(), c->d_fnch.as<uint32_t>(), c->d_ch_bad.as<uint32_t>(),
        c->d_ch_entry.as<uint64_t>(), c->d_ch_count.as<uint32_t>(), c->d_ch_exit.as<uint64_t>(),
        c->d_ch_term.as<uint32_t>(), c->d_ch_tpos.as<uint64_t>(), c->d_ch_wend.as<uint64_t>(),
        c->d_ch_aentry.as<uint64_t>(), c->d_stage.as<uint2>(), c->opts.chunk_cap, c->chunk_shift, c0, c1,
        c->d_counters.as<uint32_t>() + CNT_FIXUP, bad_cnt);
}

// Boundary discovery for chunks [c0, c1): speculative entries, chain walks
// and validation.  Host path (dev == false): kRounds validate/fixup rounds
// and a final validation, counted at val_cnt[0..kRounds], as launches of
// their own.  Device path: k_spec_entry also zeroes the run's counters (the
// k_run_init launch before), k_walk does validation round 0, and the later
// rounds run at the head of k_scan_chunks only when round 0 found an
// inconsistent chunk (launch_scan's settle): two launches where there were
// eight.
static void launch_boundary(Ctx *c, hipStream_t s, uint32_t c0, uint32_t c1, uint32_t *val_cnt, bool dev) {
    const uint32_t n = c1 - c0, cap = c->opts.chunk_cap;
    RunInit ri{nullptr, nullptr, nullptr, nullptr};
    if (dev)
        ri = RunInit{c->d_counters.as<uint32_t>(), c->d_gbase.as<uint64_t>(), c->d_blk_first.as<uint32_t>(),
                     c->d_queue.as<uint32_t>()};
    k_spec_entry<<<std::max<uint32_t>(1, nblk(n, 4)), 256, 0, s>>>(
        c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(), c->d_ch_file.as<uint32_t>() + c0,
        c->d_ch_start.as<uint64_t>() + c0, c->d_ch_end.as<uint64_t>() + c0, c->d_ch_entry.as<uint64_t>() + c0, n,
        c->opts.max_key, c->opts.spec_window, ri);
    if (!n) return;
    k_walk<<<nblk(n, 256), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(),
                                        c->d_ch_file.as<uint32_t>(), c->d_ffirst.as<uint32_t>(),
                                        c->d_fnch.as<uint32_t>(), c->d_ch_entry.as<uint64_t>(),
                                        c->d_ch_count.as<uint32_t>(), c->d_ch_exit.as<uint64_t>(),
                                        c->d_ch_term.as<uint32_t>(), c->d_ch_tpos.as<uint64_t>(),
                                        c->d_ch_wend.as<uint64_t>(), c->d_ch_aentry.as<uint64_t>(), c->d_stage.as<uint2>(),
                                        cap, c->chunk_shift, c0, c1, c->d_ch_bad.as<uint32_t>(),
                                        dev ? val_cnt : nullptr);
    if (dev) return;
    for (int r = 0; r <= kRounds; ++r) {
        k_validate<<<nblk(n, 256), 256, 0, s>>>(c->d_ch_file.as<uint32_t>(), c->d_ch_end.as<uint64_t>(),
                                                c->d_ch_entry.as<uint64_t>(), c->d_ch_exit.as<uint64_t>(),
                                                c->d_ch_term.as<uint32_t>(), c->d_ffirst.as<uint32_t>(),
                                                c->d_ch_bad.as<uint32_t>(), val_cnt + r, c0, c1,
                                                r ? val_cnt + r - 1 : nullptr);
        if (r == kRounds) break;
        launch_fixup(c, s, c0, c1, val_cnt + r);
    }
}

// Record slots of every chunk, the file summaries and, with acct (the device
// path), the run's bookkeeping: one launch of k_scan_chunks.  gbase[1] = the
// record total (clamped to cap); grng / rng as account_run.  settle (the
// device path): the validation/fixup rounds after k_walk's, when it found an
// inconsistent chunk (val = the run's CNT_VAL counters).
static void launch_scan(Ctx *c, hipStream_t s, uint64_t *gbase, uint64_t cap, bool acct, uint64_t *res = nullptr,
                        uint64_t *grng = nullptr, uint64_t *rng = nullptr, bool settle = false) {
    const uint32_t n = c->n_chunks, nb = std::max<uint32_t>(1, nblk(n, kScanBlock));
    uint32_t *cnt = c->d_counters.as<uint32_t>();
    const Settle st{c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(),
                    c->d_ch_file.as<uint32_t>(), c->d_ch_end.as<uint64_t>(), c->d_ch_bad.as<uint32_t>(),
                    c->d_ch_exit.as<uint64_t>(), c->d_ch_wend.as<uint64_t>(), c->d_ch_aentry.as<uint64_t>(),
                    c->d_stage.as<uint2>(), c->opts.chunk_cap, c->chunk_shift,
                    settle && n ? cnt + CNT_VAL : nullptr, cnt + CNT_FIXUP, cnt + CNT_BAR};
    const uint32_t grid = settle ? std::max(nb, kSettleBlocks) : nb;
    k_scan_chunks<<<grid, 64, 0, s>>>(c->d_ch_count.as<uint32_t>(), c->d_rec_base.as<uint64_t>(), n,
                                      c->d_bsum.as<uint64_t>(), gbase + 1, cap, cnt + CNT_CAP,
                                      c->d_ffirst.as<uint32_t>(), c->d_fnch.as<uint32_t>(), c->d_ch_entry.as<uint64_t>(),
                                      c->d_ch_term.as<uint32_t>(), c->d_ch_tpos.as<uint64_t>(), c->d_fterm.as<uint32_t>(),
                                      c->d_ftpos.as<uint64_t>(), c->d_ffirstrec.as<uint64_t>(), c->d_fnrec.as<uint64_t>(),
                                      c->nfiles, acct ? 1 : 0, c->d_flen.as<uint64_t>(), c->d_freset.as<uint32_t>(),
                                      c->d_carry.as<uint32_t>(), res, grng, rng, nb, st);
}

// Record table and row index (row_first) of the whole arena, one launch;
// rng = the records' range, cap = the table's records; unsettled (device
// path): the run's last settle count.
static void launch_records(Ctx *c, hipStream_t s, const uint64_t *rng, uint64_t cap, const uint32_t *unsettled) {
    const uint32_t n = c->n_chunks, ccap = c->opts.chunk_cap;
    const RowTails rt{c->d_fterm.as<uint32_t>(), c->d_ftpos.as<uint64_t>(), c->d_ffirstrec.as<uint64_t>(),
                      c->d_fnrec.as<uint64_t>(), rng, c->nfiles, c->n_rows,
                      (c->n_rows + kBlockRows - 1) / kBlockRows, unsettled};
    k_compact<<<std::max<uint32_t>(1, nblk(n, 16 * kCompactChunks)), 1024, 0, s>>>(
        c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(), c->d_ch_file.as<uint32_t>(),
        c->d_ch_wend.as<uint64_t>(), c->d_ch_entry.as<uint64_t>(), c->d_ch_aentry.as<uint64_t>(),
        c->d_ch_count.as<uint32_t>(), c->d_rec_base.as<uint64_t>(), c->d_stage.as<uint2>(), ccap, 0u, n, cap,
        c->d_rec_off.as<uint64_t>(), c->d_rec_kv.as<uint2>(), c->d_rec_file.as<uint32_t>(),
        c->d_blk_first.as<uint32_t>(), c->d_counters.as<uint32_t>(), rt);
}

// CRC partials of rows [r0, r1) (k_crc_rows; r0 a multiple of kBlockRows), block queue slot q.  Record-slot
// scratch: cap .. cap + kEpScratch; rend scratch: rows n_rows ...
static int launch_crc(Ctx *c, hipStream_t s, uint64_t r0, uint64_t r1, uint64_t cap, uint32_t q,
                      bool queue_zeroed = false) {
    if (r1 <= r0) return GCK_OK;
    const uint64_t nb = (r1 - r0 + kBlockRows - 1) / kBlockRows;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((nb + kWaves - 1) / kWaves, (uint64_t)c->n_cu);
    uint32_t *queue = c->d_queue.as<uint32_t>() + q;
    if (!queue_zeroed) GCK_HIP(hipMemsetAsync(queue, 0, 4, s));
    k_crc_rows<<<grid, kWaves * 64, 0, s>>>(
        c->arena.as<uint8_t>() + r0 * kRow, r1 - r0, c->d_blk_first.as<uint32_t>() + r0 / kBlockRows, cap,
        c->d_slice.as<uint32_t>(), c->d_nib.as<uint32_t>(), c->d_ep.as<uint2>(), c->d_rend.as<uint32_t>() + r0,
        c->d_rend.as<uint32_t>() + c->n_rows, queue, c->d_rec_off.as<uint64_t>(), c->d_rec_kv.as<uint2>(), r0
#ifdef GCK_XP_EBLK
        , c->d_ep.as<uint8_t>() + (cap + kEpScratch) * 8
#endif
        );
    return GCK_OK;
}

// mbox (the device path): the last workgroup publishes the run's counters
// there; *published tells whether a finalize was launched to do it.
static int launch_finalize(Ctx *c, hipStream_t s, const uint64_t *rng, uint64_t max_recs, uint32_t *mbox = nullptr,
                           bool *published = nullptr) {
    auto kern = c->hash_keys ? k_finalize<true> : k_finalize<false>;
    c->kd_fin_table = false;
    if (published) *published = false;
    if (!max_recs) return GCK_OK;
    // the keydir table, filled by this finalize (gck_ctx_keydir then only
    // marks and compacts), sized for the record table's capacity
    unsigned long long *ktab = nullptr;
    uint64_t kmask = 0;
    c->kd_fin_table = c->hash_keys && max_recs < kKdMaxRecs;
    if (c->kd_fin_table) {
        const uint64_t slots = kd_table_slots(kd_keys_expected(c->kd_keys_hint, max_recs));
        int rc;
        if ((rc = c->d_ktab.ensure(slots * 8 * kSlotWords)) || (rc = c->d_kdstat.ensure(12))) return rc;
        GCK_HIP(hipMemsetAsync(c->d_ktab.p, 0xFF, slots * 8 * kSlotWords, s));
        GCK_HIP(hipMemsetAsync(c->d_kdstat.p, 0, 12, s));
        c->kd_tab_slots = slots;
        ktab = c->d_ktab.as<unsigned long long>();
        kmask = slots - 1;
    }
    // one wave of workgroups that are all resident at once (a second, partial
    // round of workgroups would double the kernel's latency-bound time)
    const uint64_t want = nblk(max_recs, kFinThreads),
                   res = (uint64_t)c->n_cu * (c->hash_keys ? c->fin_blocks_per_cu_hash : c->fin_blocks_per_cu);
    const uint32_t grid = (uint32_t)(want < res ? want : res);
    kern<<<grid, kFinThreads, 0, s>>>(c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(), c->d_rec_kv.as<uint2>(),
                                    c->d_rec_file.as<uint32_t>(), c->d_fbase.as<uint64_t>(), c->d_carry.as<uint32_t>(),
                                    rng, c->d_ep.as<uint2>(), c->d_rend.as<uint32_t>(),
                                    c->d_slice.as<uint32_t>(), c->d_xinv.as<uint32_t>(),
                                    c->d_zrow.as<uint32_t>(),
                                    c->d_xa.as<uint32_t>(), c->d_xb.as<uint32_t>(),
                                    c->d_out.as<gck_rec>(), c->d_counters.as<uint32_t>(),
                                    c->hash_keys ? c->d_khash.as<uint64_t>() : nullptr, ktab, kmask,
                                    c->d_kdstat.as<uint32_t>(), mbox);
    if (published) *published = mbox != nullptr;
    return GCK_OK;
}

static int ensure_records(Ctx *c, uint64_t nr) {
    nr = nr ? nr : 1;
    int rc;
    if ((rc = c->d_rec_off.ensure(nr * 8)) || (rc = c->d_rec_kv.ensure(nr * 8)) ||
        (rc = c->d_rec_file.ensure(nr * 4)) || (rc = c->d_ep.ensure((nr + kEpScratch) * kEpBytes)) ||
        (rc = c->d_out.ensure(nr * sizeof(gck_rec))) || (c->hash_keys && (rc = c->d_khash.ensure(nr * 8))))
        return rc;
    return GCK_OK;
}

// Host bookkeeping from the per-file summaries (core/db.go:110-140): status,
// files walked, final lastOffset, records in walk order; carries if asked.
static uint64_t account_files(Ctx *c, const std::vector<uint32_t> &fterm, const std::vector<uint64_t> &ftpos,
                              const std::vector<uint64_t> &ffirst, const std::vector<uint64_t> &fnrec,
                              std::vector<uint32_t> *carry) {
    const uint32_t nf = c->nfiles;
    c->status = GCK_OK;
    c->err_file = 0;
    c->err_off = 0;
    c->files_walked = nf;
    uint64_t n_total = 0;
    uint32_t last = 0;  // keyDir.lastOffset at the start of each file
    for (uint32_t f = 0; f < nf; ++f) {
        if (carry) (*carry)[f] = last;
        const uint64_t valid = fterm[f] != T_NONE ? ftpos[f] : c->f_len[f];
        n_total = ffirst[f] + fnrec[f];
        last += (uint32_t)valid;
        if (fterm[f] == T_ERR) {  // walkFile error aborts filepath.Walk (disk.go:134-141)
            c->status = GCK_EUNEXPECTED_EOF;
            c->err_file = f;
            c->err_off = ftpos[f];
            c->files_walked = f + 1;
            break;
        }
        if (c->f_reset[f]) last = 0;  // resetOffset (core/db.go:117-119)
    }
    c->final_last_offset = last;
    return n_total;
}

static int read_file_summaries(Ctx *c, hipStream_t s, std::vector<uint32_t> &fterm, std::vector<uint64_t> &ftpos,
                               std::vector<uint64_t> &ffirst, std::vector<uint64_t> &fnrec) {
    const uint32_t nf = c->nfiles;
    fterm.assign(nf, 0);
    ftpos.assign(nf, 0);
    ffirst.assign(nf, 0);
    fnrec.assign(nf, 0);
    if (nf) {
        GCK_HIP(hipMemcpyAsync(fterm.data(), c->d_fterm.p, nf * 4, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(ftpos.data(), c->d_ftpos.p, nf * 8, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(ffirst.data(), c->d_ffirstrec.p, nf * 8, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(fnrec.data(), c->d_fnrec.p, nf * 8, hipMemcpyDeviceToHost, s));
    }
    return GCK_OK;
}

// One replay on the resident arena, every phase over all files in order, one
// host round trip after the boundary phases (exact record count, EOF
// verdicts, carries).  The CRC pass needs the record boundaries (its plan),
// and running the latency-bound boundary kernels beside an HBM-saturating
// pass slows them ~7x (loaded latency), so the phases do not overlap.
static int ctx_run_host(Ctx *c) {
    const auto t0 = std::chrono::steady_clock::now();
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint32_t nc = c->n_chunks, nf = c->nfiles;
    uint32_t *cnt = c->d_counters.as<uint32_t>();
    uint64_t *gbase = c->d_gbase.as<uint64_t>();
    GCK_HIP(hipMemsetAsync(cnt, 0, 64, s));
    GCK_HIP(hipMemsetAsync(gbase, 0, 16, s));
    GCK_HIP(hipMemsetAsync(c->d_blk_first.p, 0, 4, s));
    GCK_HIP(hipEventRecord(c->ev[PH_BOUNDARY], s));
    launch_boundary(c, s, 0, nc, cnt + CNT_VAL, false);
    GCK_HIP(hipEventRecord(c->ev[PH_SCAN], s));
    const uint64_t big_cap = ~0ull >> 1;
    launch_scan(c, s, gbase, big_cap, false);
    GCK_HIP(hipEventRecord(c->ev[PH_HOST], s));

    std::vector<uint32_t> fterm, carry(nf);
    std::vector<uint64_t> ftpos, ffirst, fnrec;
    if (read_file_summaries(c, s, fterm, ftpos, ffirst, fnrec)) return GCK_EDEVICE;
    uint32_t hcnt[16] = {};
    GCK_HIP(hipMemcpyAsync(hcnt, cnt, 64, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    // rare: inconsistencies left after the device rounds (cascading mis-speculation)
    for (uint32_t left = hcnt[CNT_VAL + kRounds]; left;) {
        launch_fixup(c, s, 0u, nc);
        GCK_HIP(hipMemsetAsync(cnt + CNT_HOSTVAL, 0, 4, s));
        k_validate<<<nblk(nc, 256), 256, 0, s>>>(c->d_ch_file.as<uint32_t>(), c->d_ch_end.as<uint64_t>(),
                                                 c->d_ch_entry.as<uint64_t>(), c->d_ch_exit.as<uint64_t>(),
                                                 c->d_ch_term.as<uint32_t>(), c->d_ffirst.as<uint32_t>(),
                                                 c->d_ch_bad.as<uint32_t>(), cnt + CNT_HOSTVAL, 0u, nc, nullptr);
        uint32_t v = 0;
        GCK_HIP(hipMemcpyAsync(&v, cnt + CNT_HOSTVAL, 4, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipStreamSynchronize(s));
        left = v;
        if (!left) {
            launch_scan(c, s, gbase, big_cap, false);
            if (read_file_summaries(c, s, fterm, ftpos, ffirst, fnrec)) return GCK_EDEVICE;
            GCK_HIP(hipMemcpyAsync(hcnt, cnt, 64, hipMemcpyDeviceToHost, s));
            GCK_HIP(hipStreamSynchronize(s));
        }
    }
    c->n_fixups = hcnt[CNT_FIXUP];
    const uint64_t n_total = account_files(c, fterm, ftpos, ffirst, fnrec, &carry);
    c->n_recs = n_total;
    if (n_total > 0xFFFFFFF0ull) return GCK_EINVAL;
    int rc;
    // capacity for the records of every file, also those after a startup
    // error (a later device-only run stages them before it learns of the error)
    const uint64_t all = nf ? std::max<uint64_t>(n_total, ffirst[nf - 1] + fnrec[nf - 1]) : n_total;
    if ((rc = ensure_records(c, all))) return rc;
    c->rec_cap = all;
    const uint64_t rng_h[2] = {0, n_total};
    if (nf) GCK_HIP(hipMemcpyAsync(c->d_carry.p, carry.data(), nf * 4, hipMemcpyHostToDevice, s));
    GCK_HIP(hipMemcpyAsync(gbase, rng_h, 16, hipMemcpyHostToDevice, s));

    GCK_HIP(hipEventRecord(c->ev[PH_RECORDS], s));
    launch_records(c, s, gbase, n_total, nullptr);
    GCK_HIP(hipEventRecord(c->ev[PH_CRC], s));
    if (n_total && (rc = launch_crc(c, s, 0, c->n_rows, n_total, kQueueCrc))) return rc;
    GCK_HIP(hipEventRecord(c->ev[PH_FINAL], s));
    if ((rc = launch_finalize(c, s, gbase, n_total))) return rc;
    GCK_HIP(hipEventRecord(c->ev[PH_END], s));
    GCK_HIP(hipMemcpyAsync(hcnt, cnt, 16, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    GCK_HIP(hipGetLastError());
    c->n_overflow = hcnt[CNT_STAGE];
    c->n_crc_fail = hcnt[CNT_REJECT];
    for (int p = 0; p < PH_NPHASE; ++p) c->ms_phase[p] = 0;
    for (int p = PH_BOUNDARY; p < PH_END; ++p) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, c->ev[p], c->ev[p + 1]);
        c->ms_phase[p] = ms;
    }
    float span = 0;
    (void)hipEventElapsedTime(&span, c->ev[PH_BOUNDARY], c->ev[PH_END]);
    c->ms_phase[PH_PIPE] = span;
    c->ms_crc_sum += c->ms_phase[PH_CRC];
    ++c->n_runs;
    c->kd_hashed = c->kd_fin_table;  // (finalize hashed the keys)
    c->kd_inserted = c->kd_fin_table;
    c->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return c->status;
}

// 32 counters / results of a run into the mapped mailbox (Ctx::h_mbox), when
// no finalize was launched to publish them
__global__ void k_publish(const uint32_t *__restrict__ cnt, uint32_t *mbox) {
    __hip_atomic_store(mbox + threadIdx.x, cnt[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The same run with no host round trip, for a context whose record table
// was sized by an earlier run (repeated replays of a resident arena): the
// bookkeeping runs on the device (k_account_grp), the record table is clamped
// to its capacity, and the counters come back through the mapped mailbox.
// Returns GCK_ERERUN when the run cannot be trusted as is (more records than
// capacity, or speculation not settled by the device rounds): the caller then
// reruns on the host path, whose result is exact.  Every phase on the one
// stream, in order: running the boundary side of later files beside the CRC
// pass of earlier ones, and the finalize of earlier rows beside the pass,
// both measured slower.
constexpr int GCK_ERERUN = -1;
static int ctx_run_device(Ctx *c) {
    const auto t0 = std::chrono::steady_clock::now();
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t m = c->stream;
    const uint64_t cap = c->rec_cap;
    const uint32_t nc = c->n_chunks;
    uint32_t *cnt = c->d_counters.as<uint32_t>();
    uint64_t *gb = c->d_gbase.as<uint64_t>();        // record base gb[0] (0) -> gb[1]
    uint64_t *grng = gb + kGbSlots, *rng = grng + 2;  // the records' range (clamped), the run's range
    uint64_t *res = c->d_counters.as<uint64_t>() + 8;
    // events: the CRC pass always (bench.py's roofline); the run's span and
    // the other phases only with phase timing on (each event between two
    // kernels costs ~5-6 us of the run, kernel trace profiles/r5a), so without
    // it ms_phase holds the CRC pass alone (gck_stats.ms_kernel documents it)
    const bool ph = c->phase_timing;
    if (ph) GCK_HIP(hipEventRecord(c->ev[PH_BOUNDARY], m));
    // six launches: speculation (+ the run's zeroing), walk (+ validation
    // round 0), scan (+ the later rounds when needed, the bookkeeping),
    // record table + row index, CRC pass, finalize (+ the mailbox)
    launch_boundary(c, m, 0, nc, cnt + CNT_VAL, true);
    if (ph) GCK_HIP(hipEventRecord(c->ev[PH_SCAN], m));
    launch_scan(c, m, gb, cap, true, res, grng, rng, true);
    if (ph) GCK_HIP(hipEventRecord(c->ev[PH_RECORDS], m));
    launch_records(c, m, grng, cap, cnt + CNT_VAL + kRounds);
    GCK_HIP(hipEventRecord(c->ev[PH_CRC], m));
    int rc;
    if ((rc = launch_crc(c, m, 0, c->n_rows, cap, kQueueCrc, true))) return rc;
    GCK_HIP(hipEventRecord(c->ev[PH_FINAL], m));
    bool published = false;
    if ((rc = launch_finalize(c, m, rng, cap, c->d_mbox, &published))) return rc;
    if (ph) GCK_HIP(hipEventRecord(c->ev[PH_END], m));
    if (!published) k_publish<<<1, 32, 0, m>>>(cnt, c->d_mbox);
    GCK_HIP(hipStreamSynchronize(m));
    GCK_HIP(hipGetLastError());
    uint32_t h[32];
    memcpy(h, c->h_mbox, 128);
    const uint64_t *hr = reinterpret_cast<const uint64_t *>(h + 16);
    if (h[CNT_VAL + kRounds] != 0 || h[CNT_CAP] != 0 || hr[5] > cap) return GCK_ERERUN;
    c->status = (int32_t)hr[0];
    c->err_file = (uint32_t)hr[1];
    c->err_off = hr[2];
    c->files_walked = (uint32_t)hr[3];
    c->final_last_offset = (uint32_t)hr[4];
    c->n_recs = hr[5];
    c->n_fixups = h[CNT_FIXUP];
    c->n_overflow = h[CNT_STAGE];
    c->n_crc_fail = h[CNT_REJECT];
    for (int p = 0; p < PH_NPHASE; ++p) c->ms_phase[p] = 0;
    auto el = [&](int a, int b) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, c->ev[a], c->ev[b]);
        return (double)ms;
    };
    if (ph) {
        c->ms_phase[PH_BOUNDARY] = el(PH_BOUNDARY, PH_SCAN);
        c->ms_phase[PH_SCAN] = el(PH_SCAN, PH_RECORDS);  // scans, file summaries, bookkeeping: one kernel
        c->ms_phase[PH_RECORDS] = el(PH_RECORDS, PH_CRC);
        c->ms_phase[PH_FINAL] = el(PH_FINAL, PH_END);
        c->ms_phase[PH_PIPE] = el(PH_BOUNDARY, PH_END);
    }
    c->ms_phase[PH_CRC] = el(PH_CRC, PH_FINAL);
    c->ms_crc_sum += c->ms_phase[PH_CRC];
    ++c->n_runs;
    c->kd_hashed = c->kd_fin_table;  // (finalize hashed the keys)
    c->kd_inserted = c->kd_fin_table;
    c->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->device_path = true;
    return c->status;
}

// gck_ctx_keydir_hash: finalize also hashes every record's key into d_khash
// (sized for the record table's capacity now; ensure_records keeps it so)
static int ctx_set_hash_keys(Ctx *c, bool on) {
    c->hash_keys = on;
    if (on && c->rec_cap) return c->d_khash.ensure(c->rec_cap * 8);
    return GCK_OK;
}

static int ctx_run(Ctx *c) {
    c->n_live = 0;  // the keydir (and its pack) belong to the previous run
    c->kd_nparts = 0;
    c->kd_valid = false;
    c->kd_hashed = false;
    c->kd_inserted = false;
    c->from_hints = false;
    if (c->rec_cap > 0 && c->nfiles > 0) {
        const int rc = ctx_run_device(c);
        if (rc != GCK_ERERUN) return rc;
        ++c->n_reruns;
    }
    c->device_path = false;
    return ctx_run_host(c);
}

}  // namespace gck

using namespace gck;

extern "C" {

int gck_ctx_create(const gck_opts *opts, gck_ctx **out) {
    if (!out) return GCK_EINVAL;
    *out = nullptr;
    gck_ctx *c = new (std::nothrow) gck_ctx();
    if (!c) return GCK_ENOMEM;
    int rc = ctx_init(&c->c, opts);
    if (rc) {
        ctx_free(&c->c);
        delete c;
        return rc;
    }
    *out = c;
    return GCK_OK;
}

void gck_ctx_destroy(gck_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->c.device);
    ctx_free(&ctx->c);
    delete ctx;
}

}  // extern "C"

int gck::ctx_load_srcs(Ctx *c, const Src *src, uint32_t nfiles) {
    std::vector<uint64_t> lens(nfiles);
    std::vector<uint8_t> reset(nfiles);
    for (uint32_t f = 0; f < nfiles; ++f) {
        if (src[f].len && !src[f].data && !src[f].path) return GCK_EINVAL;
        lens[f] = src[f].len;
        reset[f] = src[f].reset_after ? 1 : 0;
    }
    int rc = ctx_layout(c, lens.data(), nfiles, reset.data());
    if (rc) return rc;
    // pageable memory and files through the staging copier (host threads,
    // page-locked buffers), registered memory by DMA as is
    std::vector<uint8_t *> dst(nfiles);
    for (uint32_t f = 0; f < nfiles; ++f) dst[f] = c->arena.as<uint8_t>() + c->f_base[f];
    return copy_files_sync(c->device, c->stream, src, dst.data(), nfiles);
}

extern "C" {

int gck_ctx_load(gck_ctx *ctx, const gck_file *files, uint32_t nfiles) {
    if (!ctx || (nfiles && !files)) return GCK_EINVAL;
    const std::vector<Src> v = mem_srcs(files, nfiles);
    return ctx_load_srcs(&ctx->c, v.data(), nfiles);
}

int gck_ctx_keydir_hash(gck_ctx *ctx, int on) {
    if (!ctx) return GCK_EINVAL;
    if (hipSetDevice(ctx->c.device) != hipSuccess) return GCK_EDEVICE;
    return ctx_set_hash_keys(&ctx->c, on != 0);
}

int gck_ctx_run(gck_ctx *ctx) {
    if (!ctx) return GCK_EINVAL;
    return ctx_run(&ctx->c);
}

int gck_ctx_fetch(gck_ctx *ctx, gck_result *out) {
    if (!ctx || !out) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    memset(out, 0, sizeof(*out));
    out->n = c->n_recs;
    out->n_crc_fail = c->n_crc_fail;
    out->final_last_offset = c->final_last_offset;
    out->status = c->status;
    out->err_file = c->err_file;
    out->err_off = c->err_off;
    out->files_walked = c->files_walked;
    if (c->n_recs) {
        // pinned host memory: the D2H copy runs at DMA rate (and the caller
        // frees it with gck_result_free)
        GCK_HIP(hipSetDevice(c->device));
        void *h = res_alloc(c->n_recs * sizeof(gck_rec), true);
        if (!h) return GCK_ENOMEM;
        out->recs = static_cast<gck_rec *>(h);
        GCK_HIP(hipMemcpy(out->recs, c->d_out.p, c->n_recs * sizeof(gck_rec), hipMemcpyDeviceToHost));
    }
    return GCK_OK;
}

int gck_ctx_fetch_into(gck_ctx *ctx, gck_rec *dst, uint64_t cap, uint64_t *n) {
    if (!ctx || !n || (cap && !dst)) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    *n = c->n_recs;
    if (c->n_recs > cap) return GCK_EINVAL;
    if (c->n_recs) {
        GCK_HIP(hipSetDevice(c->device));
        GCK_HIP(hipMemcpy(dst, c->d_out.p, c->n_recs * sizeof(gck_rec), hipMemcpyDeviceToHost));
    }
    return GCK_OK;
}

int gck_ctx_stats(gck_ctx *ctx, gck_stats *out) {
    if (!ctx || !out) return GCK_EINVAL;
    const Ctx *c = &ctx->c;
    memset(out, 0, sizeof(*out));
    out->bytes = c->data_bytes;
    out->n_recs = c->n_recs;
    out->n_crc_fail = c->n_crc_fail;
    out->n_chunks = c->n_chunks;
    out->n_fixups = c->n_fixups;
    out->n_overflow = c->n_overflow;
    out->device_path = c->device_path ? 1u : 0u;
    out->n_reruns = c->n_reruns;
    out->ms_total = c->ms_total;
    for (int p = 0; p < PH_NPHASE && p < 12; ++p) out->ms_kernel[p] = c->ms_phase[p];
    out->status = c->status;
    out->err_file = c->err_file;
    out->err_off = c->err_off;
    out->files_walked = c->files_walked;
    out->final_last_offset = c->final_last_offset;
    out->n_files = c->nfiles;
    out->kd_longest_probe = c->kd_probe_bound > kMaxProbe ? (uint32_t)c->kd_probe_bound : 0u;
    out->n_runs = c->n_runs;
    out->ms_crc_rows_sum = c->ms_crc_sum;
    return GCK_OK;
}

int gck_ctx_phase_timing(gck_ctx *ctx, int on) {
    if (!ctx) return GCK_EINVAL;
    ctx->c.phase_timing = on != 0;
    return GCK_OK;
}

const char *gck_phase_name(int phase) {
    static const char *names[] = {"boundary", "scan", "host_sync", "records", "crc_rows",
                                  "finalize", "pipeline"};
    return phase >= 0 && phase < PH_NPHASE ? names[phase] : "";
}

int gck_ctx_device_recs(gck_ctx *ctx, const gck_rec **recs, uint64_t *n) {
    if (!ctx || !recs || !n) return GCK_EINVAL;
    *recs = ctx->c.d_out.as<gck_rec>();
    *n = ctx->c.n_recs;
    return GCK_OK;
}

void *gck_ctx_stream(gck_ctx *ctx) { return ctx ? (void *)ctx->c.stream : nullptr; }

int gck_ctx_read_file(gck_ctx *ctx, uint32_t file, uint64_t off, uint8_t *dst, uint64_t len) {
    if (!ctx || file >= ctx->c.nfiles || off + len > ctx->c.f_len[file]) return GCK_EINVAL;
    GCK_HIP(hipSetDevice(ctx->c.device));
    GCK_HIP(hipMemcpy(dst, ctx->c.arena.as<uint8_t>() + ctx->c.f_base[file] + off, len, hipMemcpyDeviceToHost));
    return GCK_OK;
}

// Host-in/host-out replay, pipelined over file groups: the files are cut into
// contiguous walk-order groups, each cut after a file that resets lastOffset
// (so every group replays exactly as the whole walk would, as shards do,
// gocask_amd/shard.py).  A ring of R device contexts holds R groups at a
// time: group g's files cross PCIe on a copy stream into context g % R, and
// it replays on the run stream as soon as they are resident, while later
// groups are still in flight; a context is laid out again for group g + R
// once group g's tuples have left.  R = G (every group resident) when the
// data-file bytes fit the budget -- gck_opts.max_resident, else 60 % of the
// device's free memory -- so a database larger than HBM streams through a
// bounded ring instead of failing (Open replays any database size,
// core/db.go:110-143; data files default to 10 GiB, db.go:45-48).  The first
// group with a startup error ends the walk (core/db.go:134-138): later groups
// contribute nothing.  The tuples of the contributing groups (file indices
// rebased) go into the caller's dst (cap records) when dst != NULL, else into
// library-owned pinned memory.
constexpr uint64_t kGroupBytes = 1ull << 30;  // smallest group target (smaller under a tight budget)
constexpr uint64_t kGroupsWanted = 4;          // groups a database is cut into when it fits
constexpr double kAutoBudgetShare = 0.6;      // share of free HBM the ring may take by default

__global__ void k_rebase_file(gck_rec *recs, uint64_t n, uint32_t base) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        recs[i].file += base;
}
// The group's tuples straight into the caller's pinned array (its device
// mapping) by the GPU's own PCIe writes, file indices rebased on the way:
// no DMA-engine copy, so it never queues behind the H2D of later groups.
// 16 B per lane; two records are 80 B = 5 uint4, the file field (bytes 8..11
// of a record) is .z of uint4 5m and .x of uint4 5m + 3.
__global__ void k_push_recs(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint64_t n_rec, uint32_t base) {
    const uint64_t bytes = n_rec * sizeof(gck_rec), n16 = bytes / 16;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i * 16 < bytes;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = src[i];
        const uint32_t m = (uint32_t)(i % 5);
        if (m == 0) v.z += base;
        if (m == 3) v.x += base;
        if (i < n16)
            dst[i] = v;
        else  // an odd record count ends 8 B into the last uint4
            *reinterpret_cast<uint2 *>(dst + i) = make_uint2(v.x, v.y);
    }
}

// Contexts of the grouped replay are kept for the next call: their arenas
// and tables stay allocated, so a repeated Open pays no hipMalloc and no table
// upload.  Bounded: at most kPoolMax contexts per device, all for one options
// key (a call with other options on that device evicts them; calls on other
// devices -- gck_replay_multi's device threads -- keep theirs).
// gck_replay_release_cache frees them.
namespace {
constexpr size_t kPoolMax = 4;
struct PoolEntry {
    gck_opts key;
    gck_ctx *ctx;
};
std::mutex g_pool_mu;
std::vector<PoolEntry> g_pool;
gck_opts pool_key(const gck_opts *o) {
    gck_opts k{};
    if (o) k = *o;
    k.max_resident = 0;  // a budget, not a context setting
    k.flags &= ~GCK_OPT_KEYS;  // a per-call output, not a context setting
    return k;
}
bool same_opts(const gck_opts &a, const gck_opts &b) {
    return a.device == b.device && a.chunk_bytes == b.chunk_bytes && a.max_key == b.max_key &&
           a.chunk_cap == b.chunk_cap && a.spec_window == b.spec_window && a.flags == b.flags;
}
int pool_take_(const gck_opts *o, gck_ctx **out) {
    const gck_opts k = pool_key(o);
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); ++i)
            if (same_opts(g_pool[i].key, k)) {
                *out = g_pool[i].ctx;
                g_pool.erase(g_pool.begin() + (ptrdiff_t)i);
                return GCK_OK;
            }
    }
    return gck_ctx_create(o, out);
}
void pool_give_(const gck_opts *o, gck_ctx *c) {
    if (!c) return;
    const gck_opts k = pool_key(o);
    std::vector<gck_ctx *> drop;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        size_t same_dev = 0;
        for (size_t i = 0; i < g_pool.size();)
            if (g_pool[i].key.device == k.device && !same_opts(g_pool[i].key, k)) {
                drop.push_back(g_pool[i].ctx);
                g_pool.erase(g_pool.begin() + (ptrdiff_t)i);
            } else {
                same_dev += g_pool[i].key.device == k.device;
                ++i;
            }
        if (same_dev < kPoolMax)
            g_pool.push_back(PoolEntry{k, c});
        else
            drop.push_back(c);
    }
    for (gck_ctx *d : drop) gck_ctx_destroy(d);
}
// device bytes held by pooled contexts for these options (reusable by a call)
uint64_t pool_bytes(const gck_opts *o) {
    const gck_opts k = pool_key(o);
    uint64_t b = 0;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto &e : g_pool)
        if (same_opts(e.key, k)) b += e.ctx->c.arena.cap;
    return b;
}
}  // namespace


void gck_replay_release_cache(void) {
    std::vector<PoolEntry> all;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        all.swap(g_pool);
    }
    for (auto &e : all) gck_ctx_destroy(e.ctx);
    stage_release();
}

// The last run's key bytes, back to back in record order, into a new pinned
// host buffer (*host, *len bytes) on the context's stream (the copy is
// complete once the stream is).
static int gather_keys(Ctx *c, void **host, uint64_t *len) {
    const uint64_t n = c->n_recs;
    const uint32_t nb = std::max<uint32_t>(1, (uint32_t)((n + kScanBlock - 1) / kScanBlock));
    hipStream_t s = c->stream;
    const size_t had = c->d_klb.cap;
    int rc;
    if ((rc = c->d_klb.ensure((nb + 2) * 8ull)) || (rc = c->d_koff.ensure((n + 1) * 8))) return rc;
    if (c->d_klb.cap != had) GCK_HIP(hipMemsetAsync(c->d_klb.p, 0, c->d_klb.cap, s));  // then self-cleaning
    k_scan_keys<<<nb, 64, 0, s>>>(c->d_rec_kv.as<uint2>(), n, c->d_koff.as<uint64_t>(), c->d_klb.as<uint64_t>());
    uint64_t tot = 0;
    GCK_HIP(hipMemcpyAsync(&tot, c->d_koff.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    if ((rc = c->d_keyblob.ensure(tot ? tot : 1))) return rc;
    k_gather_keys<<<(uint32_t)c->n_cu * 4, 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(),
                                                        c->d_rec_kv.as<uint2>(), c->d_koff.as<uint64_t>(), n,
                                                        c->d_keyblob.as<uint8_t>());
    if (hipHostMalloc(host, tot ? tot : 1, hipHostMallocDefault) != hipSuccess) {
        *host = nullptr;
        return GCK_ENOMEM;
    }
    *len = tot;
    if (tot) GCK_HIP(hipMemcpyAsync(*host, c->d_keyblob.p, tot, hipMemcpyDeviceToHost, s));
    return GCK_OK;
}

// The live entries of the context's last gck_kd_merge shaped on the device as
// the host wants them (gck_rec array; with want_keys the keys back to back,
// unpadded) -- mo_sizes first (the key bytes), then mo_out into
// host memory.  (The host had copied the 64-byte entries and padded keys out
// and rebuilt both arrays entry by entry: ~0.25 s of a C3 live Open,
// profiles/r6n.)
static int mo_sizes(Ctx *c, bool want_keys, uint64_t *n, uint64_t *key_bytes) {
    *n = c->n_merged;
    *key_bytes = 0;
    if (!c->n_merged || !want_keys) return GCK_OK;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint64_t m = c->n_merged;
    const uint32_t nb = std::max<uint32_t>(1, (uint32_t)((m + kScanBlock - 1) / kScanBlock));
    const size_t had = c->d_klb.cap;
    int rc;
    if ((rc = c->d_klb.ensure((nb + 2) * 8ull)) || (rc = c->d_koff.ensure((m + 1) * 8))) return rc;
    if (c->d_klb.cap != had) GCK_HIP(hipMemsetAsync(c->d_klb.p, 0, c->d_klb.cap, s));  // then self-cleaning
    k_mo_scan<<<nb, 64, 0, s>>>(c->d_mhdr.as<gck_kd_entry>(), m, c->d_koff.as<uint64_t>(), c->d_klb.as<uint64_t>());
    GCK_HIP(hipMemcpyAsync(key_bytes, c->d_koff.as<uint64_t>() + m, 8, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    return GCK_OK;
}
static int mo_out(Ctx *c, gck_rec *h, uint8_t *keys, uint64_t key_bytes) {
    const uint64_t m = c->n_merged;
    if (!m) return GCK_OK;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = c->d_mout.ensure(m * sizeof(gck_rec))) || (keys && (rc = c->d_keyblob.ensure(key_bytes ? key_bytes : 1))))
        return rc;
    k_mo_out<<<(uint32_t)c->n_cu * 4, 256, 0, s>>>(c->d_mhdr.as<gck_kd_entry>(), c->d_mkeys.as<uint8_t>(),
                                                   c->d_koff.as<uint64_t>(), m, c->d_mout.as<gck_rec>(),
                                                   keys ? c->d_keyblob.as<uint8_t>() : nullptr);
    GCK_HIP(hipMemcpyAsync(h, c->d_mout.p, m * sizeof(gck_rec), hipMemcpyDeviceToHost, s));
    if (keys && key_bytes) GCK_HIP(hipMemcpyAsync(keys, c->d_keyblob.p, key_bytes, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    return GCK_OK;
}

// sink: gck_replay_multi's hook (GroupSink, gck_internal.h): each group's
// context is handed to it after the group has replayed, and no tuples or keys
// are delivered (out carries the outcome only).
static int replay_grouped(const Src *files, uint32_t nfiles, const gck_opts *opts, bool into, gck_rec *dst,
                          uint64_t cap, gck_result *out, GroupSink *sink = nullptr) {
    const auto t_call = std::chrono::steady_clock::now();
    memset(out, 0, sizeof(*out));
    for (uint32_t f = 0; f < nfiles; ++f)
        if (files[f].len && !files[f].data && !files[f].path) return GCK_EINVAL;
    const uint64_t budget_opt = opts ? opts->max_resident : 0;
    int rc0 = GCK_OK;
    // group target: about a quarter of the database (at least kGroupBytes),
    // or a third of a tight budget (so at least two groups of files smaller
    // than that fit at once).  Few groups: each is a device context, and
    // creating 16 of them took 0.25-0.34 s of a 1.1 s Open of C3, while the
    // replay a group hides under the next group's copy is ~100x shorter than
    // that copy anyway.
    uint64_t all_bytes = 0;
    for (uint32_t f = 0; f < nfiles; ++f) all_bytes += files[f].len;
    const uint64_t want = std::max<uint64_t>(kGroupBytes, all_bytes / kGroupsWanted);
    const uint64_t tgt = budget_opt ? std::max<uint64_t>(1, std::min(want, budget_opt / 3)) : want;
    std::vector<uint32_t> cut{0};  // group g = files [cut[g], cut[g+1])
    {
        uint64_t acc = 0;
        for (uint32_t f = 0; f < nfiles; ++f) {
            acc += files[f].len;
            if (acc >= tgt && files[f].reset_after && f + 1 < nfiles) {
                cut.push_back(f + 1);
                acc = 0;
            }
        }
    }
    cut.push_back(nfiles);
    const uint32_t G = (uint32_t)cut.size() - 1;
    std::vector<uint64_t> gbytes(G, 0);
    for (uint32_t g = 0; g < G; ++g)
        for (uint32_t f = cut[g]; f < cut[g + 1]; ++f) gbytes[g] += (files[f].len + kRow - 1) / kRow * kRow;
    const uint64_t maxg = std::max<uint64_t>(*std::max_element(gbytes.begin(), gbytes.end()), kRow);
    // ring size R: every group when the bytes fit the budget
    uint64_t budget = budget_opt;
    if (!budget && (rc0 = auto_budget(opts, &budget))) return rc0;
    const auto t_budget = std::chrono::steady_clock::now();  // (the process's first Open: HIP's initialisation)
    // a sink (gck_replay_multi, GCK_OPT_LIVE) keeps each group's packed
    // keydir on the device until the exchange: an eighth of the budget is
    // left for those (C3: packs are ~1 % of the data bytes; a database of
    // records under ~600 B can need more, and its pack allocation then fails
    // with GCK_ENOMEM as a group that does not fit does)
    if (sink) budget -= budget / 8;
    uint64_t fit = 0;
    for (uint32_t g = 0; g < G; ++g) fit += gbytes[g];
    const uint32_t R = fit <= budget ? G : (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(G, budget / maxg));
    out->n_groups = G;
    out->n_resident = R;
    std::vector<gck_ctx *> cs(R, nullptr);
    std::vector<hipEvent_t> ev(G, nullptr);
    hipStream_t copy = nullptr, run_s = nullptr;
    std::vector<hipStream_t> own_s(R, nullptr);  // the contexts' own streams while they run on run_s
    std::vector<void *> chunks(G, nullptr);        // ring mode, gck_replay: each group's tuples (pinned)
    std::vector<uint64_t> chunk_n(G, 0);
    const bool want_keys = !sink && opts && (opts->flags & GCK_OPT_KEYS);
    if (sink) into = false;
    std::vector<void *> kchunks(G, nullptr);  // GCK_OPT_KEYS: each group's key bytes (pinned)
    std::vector<uint64_t> kchunk_n(G, 0);
    int rc = GCK_OK;
    Copier cp;  // the file copies (staging.hip)
    auto cleanup = [&](bool keep) {
        (void)cp.finish();
        if (copy) (void)hipStreamSynchronize(copy);
        if (run_s) {
            (void)hipStreamSynchronize(run_s);
            for (uint32_t k = 0; k < R; ++k)
                if (own_s[k]) cs[k]->c.stream = own_s[k];
            (void)hipStreamDestroy(run_s);
        }
        for (auto *c : cs)
            if (c) (void)hipStreamSynchronize(c->c.stream);
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        if (copy) (void)hipStreamDestroy(copy);
        // (after the stream synchronisations: a key gather's D2H may still be
        // writing a kchunk on an error path)
        for (void *q : kchunks)
            if (q) (void)hipHostFree(q);
        for (void *p : chunks)
            if (p) (void)hipHostFree(p);
        for (auto *c : cs) {
            if (!c) continue;
            if (keep)
                pool_give_(opts, c);
            else
                gck_ctx_destroy(c);
        }
    };
    // the staging buffers (pinned host memory, 0.15-0.25 s for 0.5-1 GiB on a
    // process's first Open) are allocated on a helper thread while the
    // contexts are created
    int pre_rc = GCK_OK;
    std::thread pre([&] { pre_rc = stage_prealloc(opts ? opts->device : 0, stage_buffers_wanted()); });
    // the contexts on threads of their own: a fresh process's first ones
    // create the device's hardware queues and load the code objects
    {
        std::vector<int> trc(R, GCK_OK);
        std::vector<std::thread> th;
        for (uint32_t k = 1; k < R; ++k) th.emplace_back([&, k] { trc[k] = pool_take_(opts, &cs[k]); });
        trc[0] = pool_take_(opts, &cs[0]);
        for (auto &t : th) t.join();
        for (uint32_t k = 0; k < R && !rc; ++k) rc = trc[k];
    }
    const auto t_taken = std::chrono::steady_clock::now();
    pre.join();
    if (!rc) rc = pre_rc == GCK_ENOMEM ? GCK_OK : pre_rc;  // (the copier retries the allocation)
    if (rc) {
        cleanup(true);
        return rc;
    }
    const auto t_ctx = std::chrono::steady_clock::now();
    const int dev = cs[0]->c.device;
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&copy, hipStreamNonBlocking) != hipSuccess) {
        cleanup(false);
        return GCK_EDEVICE;
    }
    // Every group runs on ONE stream, created right after the copy stream.
    // Streams beyond the device's hardware queues share them in order, and a
    // group stream that shared the copy stream's queue would sit behind every
    // queued file copy; two streams map to two queues.
    if (hipStreamCreateWithFlags(&run_s, hipStreamNonBlocking) != hipSuccess) {
        cleanup(false);
        return GCK_EDEVICE;
    }
    for (uint32_t k = 0; k < R; ++k) {
        own_s[k] = cs[k]->c.stream;
        cs[k]->c.stream = run_s;
    }
    if ((rc = cp.start(dev, copy, &ev))) {
        cleanup(false);
        return rc;
    }
    // caller memory that is page-locked (gck_host_register) goes by DMA as is
    std::vector<uint8_t> pinned(nfiles, 0);
    for (uint32_t f = 0; f < nfiles; ++f) pinned[f] = files[f].data && files[f].len && host_pinned(files[f].data);
    const bool trace = getenv("GCK_REPLAY_TRACE") != nullptr;
    const auto t_begin = std::chrono::steady_clock::now();
    if (trace)
        fprintf(stderr,
                "[gck_replay] budget (HIP up) at %.2f ms, %u contexts taken at %.2f ms, staging ready (contexts ready) at "
                "%.2f ms, copier started at %.2f ms after the call\n",
                std::chrono::duration<double, std::milli>(t_budget - t_call).count(), R,
                std::chrono::duration<double, std::milli>(t_taken - t_call).count(),
                std::chrono::duration<double, std::milli>(t_ctx - t_call).count(),
                std::chrono::duration<double, std::milli>(t_begin - t_call).count());
    hipEvent_t tev0 = nullptr;
    if (trace) {
        (void)hipEventCreate(&tev0);
        (void)hipEventRecord(tev0, copy);
    }
    // lay group g out in its ring context and queue its files' H2D
    auto prep = [&](uint32_t g) -> int {
        Ctx *c = &cs[g % R]->c;
        const uint32_t f0 = cut[g], n = cut[g + 1] - f0;
        std::vector<uint64_t> lens(n);
        std::vector<uint8_t> reset(n);
        for (uint32_t k = 0; k < n; ++k) {
            lens[k] = files[f0 + k].len;
            reset[k] = files[f0 + k].reset_after ? 1 : 0;
        }
        int r;
        if ((r = ctx_layout(c, lens.data(), n, reset.data()))) return r;
        // a fresh context would take the host path on its first run, whose
        // small D2H copies queue behind the file copies: give it a record table
        // for the device path (one record per 256 B; more reruns exactly)
        uint64_t bytes = 0;
        for (uint32_t k = 0; k < n; ++k) bytes += lens[k];
        const uint64_t est = bytes / 256 + 4096;
        if (c->rec_cap < est) {
            if ((r = ensure_records(c, est))) return r;
            c->rec_cap = est;
        }
        if (hipEventCreateWithFlags(&ev[g], trace ? hipEventDefault : hipEventDisableTiming) != hipSuccess)
            return GCK_EDEVICE;
        for (uint32_t k = 0; k < n; ++k) {
            const Src &f = files[f0 + k];
            uint8_t *d = c->arena.as<uint8_t>() + c->f_base[k];
            if (!f.len) continue;
            if (pinned[f0 + k]) {
                if ((r = cp.direct(f.data, f.len, d))) return r;
            } else {
                cp.add(g, f, 0, f.len, d);
            }
        }
        cp.seal(g);  // its event follows its last chunk on the copy stream
        return GCK_OK;
    };
    // every resident group's layout first, then (in prep) its copies: a
    // layout uploads its tables by a kernel, never behind the file copies
    for (uint32_t g = 0; g < std::min(R, G) && !rc; ++g) rc = prep(g);
    uint32_t last = G;  // groups [0, last) contribute
    uint64_t off = 0;
    bool early = into;  // tuples delivered group by group while the caller's array has room
    // the device mapping of a registered (pinned) dst, for k_push_recs; plain
    // pageable memory has none and takes the DMA copy
    gck_rec *ddst = nullptr;
    if (into && dst && cap) {
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, dst, 0) == hipSuccess && dp) ddst = static_cast<gck_rec *>(dp);
        else (void)hipGetLastError();
    }
    uint64_t n_total = 0;
    std::vector<uint64_t> g_fail(G, 0);
    int32_t st_status = GCK_OK;
    uint32_t st_err_file = 0, st_walked = 0, st_last = 0;
    uint64_t st_err_off = 0;
    for (uint32_t g = 0; g < G && !rc; ++g) {
        Ctx *c = &cs[g % R]->c;
        if ((rc = cp.wait_recorded(g))) break;
        if (hipStreamWaitEvent(c->stream, ev[g], 0) != hipSuccess) {
            rc = GCK_EDEVICE;
            break;
        }
        const auto tr0 = std::chrono::steady_clock::now();
        // a sink builds each group's keydir: its keys are hashed in the
        // group's finalize pass (gck_ctx_keydir then reads no key for them)
        if (int hr = ctx_set_hash_keys(c, sink != nullptr)) {
            rc = hr;
            break;
        }
        const int r = ctx_run(c);
        if (trace)
            fprintf(stderr, "[gck_replay] group %u (slot %u) run returned at %.2f ms (run call %.2f ms, device path %d)\n",
                    g, g % R, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_begin).count(),
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count(),
                    (int)c->device_path);
        if (r != GCK_OK && r != GCK_EUNEXPECTED_EOF) {
            rc = r;
            break;
        }
        if (want_keys && c->n_recs && (rc = gather_keys(c, &kchunks[g], &kchunk_n[g]))) break;
        if (sink && (rc = sink->group(g, cut[g], cs[g % R]))) break;
        g_fail[g] = c->n_crc_fail;
        n_total += c->n_recs;
        st_status = c->status;
        st_err_file = cut[g] + c->err_file;
        st_err_off = c->err_off;
        st_walked = cut[g] + c->files_walked;
        st_last = c->final_last_offset;  // cuts follow resetting files: the last contributing group's
        if (c->n_recs && early) {
            if (off + c->n_recs > cap) {
                early = false;
            } else if (ddst) {
                k_push_recs<<<(uint32_t)c->n_cu * 4, 256, 0, c->stream>>>(c->d_out.as<uint4>(),
                                                                         reinterpret_cast<uint4 *>(ddst + off),
                                                                         c->n_recs, cut[g]);
                off += c->n_recs;
            } else {
                if (cut[g])
                    k_rebase_file<<<(uint32_t)c->n_cu * 4, 256, 0, c->stream>>>(c->d_out.as<gck_rec>(), c->n_recs, cut[g]);
                if (hipMemcpyAsync(dst + off, c->d_out.p, c->n_recs * sizeof(gck_rec), hipMemcpyDeviceToHost,
                                   c->stream) != hipSuccess)
                    rc = GCK_EDEVICE;
                off += c->n_recs;
            }
        } else if (c->n_recs && !into && !sink) {
            // library-owned output: the group's tuples into a pinned chunk now
            // (written by the GPU through its mapping while later groups still
            // copy; in ring mode the context is about to be reused), joined by
            // the host at the end
            void *hp = nullptr, *dp = nullptr;
            if (hipHostMalloc(&hp, c->n_recs * sizeof(gck_rec), hipHostMallocMapped) != hipSuccess ||
                hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess) {
                if (hp) (void)hipHostFree(hp);
                rc = GCK_ENOMEM;
                break;
            }
            chunks[g] = hp;
            chunk_n[g] = c->n_recs;
            k_push_recs<<<(uint32_t)c->n_cu * 4, 256, 0, c->stream>>>(c->d_out.as<uint4>(), static_cast<uint4 *>(dp),
                                                                     c->n_recs, cut[g]);
        }
        if (r == GCK_EUNEXPECTED_EOF) {
            last = g + 1;
            break;
        }
        if (g + R < G) {  // this context takes group g + R once its tuples have left
            if (hipStreamSynchronize(c->stream) != hipSuccess) {
                rc = GCK_EDEVICE;
                break;
            }
            rc = prep(g + R);
        }
    }
    if (rc) {
        cleanup(false);
        return rc;
    }
    if (trace) {
        (void)hipStreamSynchronize(run_s);
        (void)hipStreamSynchronize(copy);
        const double host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_begin).count();
        float copy_ms = 0;
        (void)hipEventElapsedTime(&copy_ms, tev0, ev[last - 1]);
        fprintf(stderr, "[gck_replay] groups %u resident %u host %.2f ms, H2D (copy stream) %.2f ms\n", G, R, host_ms,
                copy_ms);
        (void)hipEventDestroy(tev0);
    }
    out->n = n_total;
    out->status = st_status;
    out->err_file = st_err_file;
    out->err_off = st_err_off;
    out->files_walked = st_walked;
    out->final_last_offset = st_last;
    for (uint32_t g = 0; g < last; ++g) out->n_crc_fail += g_fail[g];
    if (want_keys) {  // the groups' key bytes, in order
        uint64_t kt = 0;
        std::vector<std::pair<const void *, uint64_t>> segs;
        for (uint32_t g = 0; g < last; ++g) {
            kt += kchunk_n[g];
            if (kchunk_n[g]) segs.emplace_back(kchunks[g], kchunk_n[g]);
        }
        if (hipStreamSynchronize(run_s) != hipSuccess) {
            cleanup(false);
            return GCK_EDEVICE;
        }
        void *kp = res_alloc(kt, false);
        if (!kp) {
            cleanup(true);
            return GCK_ENOMEM;
        }
        par_gather(static_cast<uint8_t *>(kp), segs);
        out->keys = static_cast<uint8_t *>(kp);
        out->keys_len = kt;
    }
    auto drop_keys = [&]() {  // an error return hands back no key blob
        res_free(out->keys);
        out->keys = nullptr;
        out->keys_len = 0;
    };
    if (into) {
        cleanup(true);
        if (cap < n_total) {  // out->n says how many records to make room for
            drop_keys();
            return GCK_EINVAL;
        }
        return out->status;
    }
    if (sink) {  // the outcome only: the sink took what it needed from each group
        out->n = 0;
        cleanup(true);
        return out->status;
    }
    // the groups' pinned chunks into one plain array, in order
    if (hipStreamSynchronize(run_s) != hipSuccess) {
        cleanup(false);
        drop_keys();
        return GCK_EDEVICE;
    }
    gck_rec *h = nullptr;
    if (n_total) {
        h = static_cast<gck_rec *>(res_alloc(n_total * sizeof(gck_rec), false));
        if (!h) {
            cleanup(true);
            drop_keys();
            return GCK_ENOMEM;
        }
        std::vector<std::pair<const void *, uint64_t>> segs;
        for (uint32_t g = 0; g < last; ++g)
            if (chunk_n[g]) segs.emplace_back(chunks[g], chunk_n[g] * sizeof(gck_rec));
        par_gather(reinterpret_cast<uint8_t *>(h), segs);
    }
    out->recs = h;
    if (trace)
        fprintf(stderr, "[gck_replay] results in host memory at %.2f ms after the call\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count());
    cleanup(true);
    return out->status;
}

// GCK_OPT_LIVE: the live keydir instead of every record -- each file group's
// device keydir (tombstones kept) packed as it finishes, then merged in walk
// order on the device: gck_replay_multi's path with the one device of the
// options (no RCCL: every pair is a device copy).
static bool want_live(const gck_opts *o) { return o && (o->flags & GCK_OPT_LIVE); }
static int replay_live(const Src *v, uint32_t nfiles, const gck_opts *opts, gck_result *out) {
    return replay_multi(v, nfiles, std::vector<int>{opts->device}, opts, out, false);
}

int gck_replay(const gck_file *files, uint32_t nfiles, const gck_opts *opts, gck_result *out) {
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    if (nfiles && !files) return GCK_EINVAL;
    const std::vector<Src> v = mem_srcs(files, nfiles);
    if (want_live(opts)) return replay_live(v.data(), nfiles, opts, out);
    return replay_grouped(v.data(), nfiles, opts, false, nullptr, 0, out);
}

int gck_replay_into(const gck_file *files, uint32_t nfiles, const gck_opts *opts, gck_rec *dst, uint64_t cap,
                    gck_result *out) {
    if (!out || (cap && !dst) || (nfiles && !files)) return GCK_EINVAL;
    const std::vector<Src> v = mem_srcs(files, nfiles);
    if (want_live(opts)) {
        memset(out, 0, sizeof(*out));
        const int rc = replay_live(v.data(), nfiles, opts, out);
        if (rc != GCK_OK && rc != GCK_EUNEXPECTED_EOF) return rc;
        gck_rec *h = out->recs;
        out->recs = nullptr;
        if (out->n > cap) {
            res_free(h);
            res_free(out->keys);
            out->keys = nullptr;
            out->keys_len = 0;
            return GCK_EINVAL;
        }
        if (out->n) memcpy(dst, h, out->n * sizeof(gck_rec));
        res_free(h);
        return rc;
    }
    return replay_grouped(v.data(), nfiles, opts, true, dst, cap, out);
}

int gck_replay_paths(const gck_path *files, uint32_t nfiles, const gck_opts *opts, gck_result *out) {
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    if (nfiles && !files) return GCK_EINVAL;
    std::vector<Src> v;
    int rc = open_srcs(files, nfiles, v);
    if (rc) return rc;
    rc = want_live(opts) ? replay_live(v.data(), nfiles, opts, out)
                         : replay_grouped(v.data(), nfiles, opts, false, nullptr, 0, out);
    close_srcs(v);
    return rc;
}

void gck_result_free(gck_result *res) {
    if (!res) return;
    res_free(res->recs);
    res_free(res->keys);
    res->recs = nullptr;
    res->keys = nullptr;
    res->n = 0;
    res->keys_len = 0;
}

int gck_host_register(const void *p, uint64_t len) {
    if (!p || !len) return GCK_EINVAL;
    GCK_HIP(hipHostRegister(const_cast<void *>(p), len, hipHostRegisterDefault));
    return GCK_OK;
}

int gck_host_unregister(const void *p) {
    if (!p) return GCK_EINVAL;
    GCK_HIP(hipHostUnregister(const_cast<void *>(p)));
    return GCK_OK;
}

int gck_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *gck_version(void) { return "gocask_hip 0.1 (gfx950)"; }

const char *gck_last_error(void) { return gck::last_error(); }

}  // extern "C"

namespace gck {
// The data bytes a ring may hold when max_resident is 0: a share of the
// device's free memory plus the arenas pooled for these options (records,
// stage and output add about a third to the data bytes).
int auto_budget(const gck_opts *opts, uint64_t *budget) {
    size_t fr = 0, tt = 0;
    if (hipSetDevice(opts ? opts->device : 0) != hipSuccess || hipMemGetInfo(&fr, &tt) != hipSuccess) {
        (void)hipGetLastError();
        return GCK_EDEVICE;
    }
    *budget = (uint64_t)(kAutoBudgetShare * (double)(fr + pool_bytes(opts)) / 1.35);
    return GCK_OK;
}
int replay_groups_to(const Src *files, uint32_t nfiles, const gck_opts *opts, GroupSink *sink, gck_result *out) {
    if (!out || !sink || (nfiles && !files)) return GCK_EINVAL;
    return replay_grouped(files, nfiles, opts, false, nullptr, 0, out, sink);
}
int pool_take(const gck_opts *o, gck_ctx **out) { return pool_take_(o, out); }
void pool_give(const gck_opts *o, gck_ctx *c) { pool_give_(o, c); }
int ctx_gather_keys(Ctx *c, void **host, uint64_t *len) { return gather_keys(c, host, len); }
int merged_out_sizes(Ctx *c, bool want_keys, uint64_t *n, uint64_t *key_bytes) {
    return mo_sizes(c, want_keys, n, key_bytes);
}
int merged_out(Ctx *c, gck_rec *h, uint8_t *keys, uint64_t key_bytes) { return mo_out(c, h, keys, key_bytes); }
}  // namespace gck

extern "C" {

#ifdef GCK_CLOCK_STAMPS
// Diagnostic build only: which 0 = k_crc_rows' stamps of the last run, 1 =
// k_clk_stream's; out receives 4 u64 per wavefront (clock, real time at the
// loop start, then at the end), kClkWaves entries; zeroed by reset.
int gck_xp_clock_reset(void) {
    void *p = nullptr;
    GCK_HIP(hipGetSymbolAddress(&p, HIP_SYMBOL(g_clk)));
    GCK_HIP(hipMemset(p, 0, sizeof(uint64_t) * kClkKinds * 4 * kClkWaves));
    return GCK_OK;
}
// wavefronts each kind's stamps hold (the readers size their buffers by it)
int gck_xp_clock_waves(void) { return (int)kClkWaves; }
int gck_xp_clock_read(int which, uint64_t *out) {
    if (which < 0 || which >= kClkKinds || !out) return GCK_EINVAL;
    GCK_HIP(hipDeviceSynchronize());
    GCK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk), sizeof(uint64_t) * 4 * kClkWaves,
                                sizeof(uint64_t) * 4 * kClkWaves * which));
    return GCK_OK;
}
// k_finalize's per-wavefront (load wait, compute) shader cycles of the last run
int gck_xp_fin_split(uint64_t *out) {
    if (!out) return GCK_EINVAL;
    GCK_HIP(hipDeviceSynchronize());
    GCK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fin_split), sizeof(uint64_t) * 2 * kClkWaves, 0));
    return GCK_OK;
}
// the XCC id of each stamped wavefront (kClkWaves entries)
int gck_xp_clock_xcc(int which, uint32_t *out) {
    if (which < 0 || which >= kClkKinds || !out) return GCK_EINVAL;
    GCK_HIP(hipDeviceSynchronize());
    GCK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk_xcc), sizeof(uint32_t) * kClkWaves,
                                sizeof(uint32_t) * kClkWaves * which));
    return GCK_OK;
}
// iters back-to-back stamped stream reads of the context's arena; *ms = per launch
int gck_xp_clock_stream(gck_ctx *ctx, int iters, double *ms) {
    if (!ctx || iters <= 0) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    GCK_HIP(hipSetDevice(c->device));
    const uint64_t n16 = c->arena_len / 16;
    if (!n16) return GCK_EINVAL;
    const uint32_t grid = (uint32_t)c->n_cu * 8;
    uint32_t *sink = c->d_counters.as<uint32_t>() + 14;
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    GCK_HIP(hipEventRecord(a, c->stream));
    for (int i = 0; i < iters; ++i) k_clk_stream<<<grid, 256, 0, c->stream>>>(c->arena.as<uint4>(), n16, sink);
    GCK_HIP(hipEventRecord(b, c->stream));
    GCK_HIP(hipEventSynchronize(b));
    float t = 0;
    GCK_HIP(hipEventElapsedTime(&t, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (ms) *ms = t / iters;
    return GCK_OK;
}
#endif

}  // extern "C"

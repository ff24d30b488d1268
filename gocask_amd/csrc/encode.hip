// encode.hip — device record encoder for bulk corpus builds.
//
// Writes records byte-for-byte as the reference's write path does:
//   Put:    header{CRC32(val), t, len(key), len(val)} || key || val
//           (core/db.go:185-212, serializeEntry core/db.go:272-284,
//            newKVHeader core/header.go:18-28, encode core/header.go:38-48)
//   Delete: header{CRC32(key), t, 0, len(key)} || key      (core/db.go:245-247)
//   Rotate: new file when size + entrySize > MaxDataFileSize (core/db.go:214-232),
//           named data_<n>_<unix>.csk (internal/fs/disk.go:71-82).
// The op stream is the synthetic corpus spec of DESIGN.md "Corpus"; the host
// plans offsets (a sequential rotation rule), the device writes the bytes and
// computes each CRC.  tests/ cross-check it against the oracle's CPU generator.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "gck_internal.h"
#include "gck_crc_wave.h"

namespace gck {

constexpr uint32_t kZipfN = 65473;

// Built once per process by a function-local static's initializer, which C++
// runs exactly once even when several threads encode at once (bench.py
// --lib-multi encodes a corpus per device from one thread each; a lazily
// filled vector let a second thread sample a half-built table: a different
// corpus, now and then).
static const std::vector<uint32_t> &zipf_thr() {
    static const std::vector<uint32_t> thr = [] {
        std::vector<double> cum(kZipfN);
        double acc = 0.0;
        for (uint32_t r = 1; r <= kZipfN; ++r) {
            acc += std::pow((double)r, -1.1);
            cum[r - 1] = acc;
        }
        std::vector<uint32_t> t(kZipfN - 1);
        for (uint32_t k = 0; k + 1 < kZipfN; ++k) {
            const double v = std::floor(cum[k] / acc * 4294967296.0);
            t[k] = v >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)v;
        }
        return t;
    }();
    return thr;
}

static uint32_t zipf_sample(const std::vector<uint32_t> &thr, uint32_t u) {
    // r = 1 + #{k : thr[k] <= u}
    return 1u + (uint32_t)(std::upper_bound(thr.begin(), thr.end(), u) - thr.begin());
}

struct OpDesc {
    uint64_t dst;    // arena offset of the record
    uint64_t keyid;
    uint32_t vlen;
    uint32_t klen;   // bit 31: tombstone
};

// One lane per op: key, value (generated, CRC'd on the fly, optionally one bit
// flipped after the CRC), then the header.
__global__ __launch_bounds__(256) void k_encode(uint8_t *__restrict__ arena, const OpDesc *__restrict__ ops,
                                                uint64_t n_ops, uint64_t seed, uint64_t kseed, uint32_t ts_base,
                                                uint32_t flip_permille) {
    __shared__ uint32_t T[256];
    for (uint32_t n = threadIdx.x; n < 256; n += blockDim.x) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
        T[n] = c;
    }
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_ops) return;
    const OpDesc o = ops[i];
    const bool tomb = (o.klen >> 31) != 0;
    const uint32_t klen = o.klen & 0x7FFFFFFFu, vlen = o.vlen;
    uint8_t *p = arena + o.dst;
    uint8_t *key = p + 16;
    const uint64_t w0 = mix64(o.keyid ^ H(kseed, 7, 0));
    uint32_t kc = 0xFFFFFFFFu;
    for (uint32_t j = 0; j < klen; ++j) {
        const uint64_t w = j < 8 ? w0 : H(kseed, 8, o.keyid * 64 + j / 8);
        const uint8_t b = (uint8_t)(w >> (8 * (j % 8)));
        key[j] = b;
        kc = T[(kc ^ b) & 0xff] ^ (kc >> 8);
    }
    uint32_t crc, ks;
    if (tomb) {
        crc = ~kc;
        ks = 0;
    } else {
        uint8_t *v = key + klen;
        uint64_t flip_byte = ~0ull;
        uint8_t flip_mask = 0;
        if (flip_permille && vlen && (H(seed, 4, i) % 1000u) < flip_permille) {
            const uint64_t bit = H(seed, 9, i) % (8ull * vlen);
            flip_byte = bit / 8;
            flip_mask = (uint8_t)(1u << (bit % 8));
        }
        uint32_t c = 0xFFFFFFFFu;
        for (uint32_t j = 0; j < vlen; j += 8) {
            const uint64_t w = H(seed, 5, (i << 20) | (j / 8));
            const uint32_t nb = vlen - j < 8 ? vlen - j : 8;
            for (uint32_t b = 0; b < nb; ++b) {
                const uint8_t x = (uint8_t)(w >> (8 * b));
                c = T[(c ^ x) & 0xff] ^ (c >> 8);
                v[j + b] = (j + b == flip_byte) ? (uint8_t)(x ^ flip_mask) : x;
            }
        }
        crc = ~c;
        ks = klen;
    }
    const uint32_t ts = ts_base + (uint32_t)i;
    const uint32_t hv[4] = {crc, ts, ks, vlen};
    for (int k = 0; k < 16; ++k) p[k] = (uint8_t)(hv[k / 4] >> (8 * (k % 4)));
}

// Host plan: op sizes from the spec, greedy rotation, lexical walk order.
// Keys: from cfg->seed, or with key_seed from one universe shared by the
// per-file corpora of gck_encode_files (kfile = the file's id).
static uint64_t key_seed_of(const gck_corpus_cfg *cfg) { return cfg->key_seed ? cfg->key_seed : cfg->seed; }
static int plan(const gck_corpus_cfg *cfg, uint64_t kfile, std::vector<OpDesc> &ops, std::vector<uint32_t> &op_file,
                std::vector<uint64_t> &sizes) {
    if (cfg->key_min < 8 || cfg->key_max > 512 || cfg->key_max < cfg->key_min) return GCK_EINVAL;
    if (!cfg->n_ops && !cfg->n_files) return GCK_EINVAL;
    if (!cfg->val_fixed && cfg->max_file_size == 0) return GCK_EINVAL;
    if (cfg->val_fixed >= (1u << 23)) return GCK_EINVAL;
    const auto &thr = zipf_thr();
    const uint64_t kseed = key_seed_of(cfg);
    uint32_t cur = 0;
    uint64_t size = 0;
    sizes.clear();
    for (uint64_t i = 0;; ++i) {
        if (cfg->n_ops && i >= cfg->n_ops) break;
        const bool tomb = cfg->tomb_permille && (H(cfg->seed, 3, i) % 1000u) < cfg->tomb_permille;
        const uint64_t kidx = cfg->key_seed ? (kfile << 32 | i) : i;
        const uint64_t keyid = cfg->key_universe ? H(kseed, 1, kidx) % cfg->key_universe : kidx;
        const uint32_t klen =
            cfg->key_min +
            (cfg->key_max > cfg->key_min ? (uint32_t)(H(kseed, 6, keyid) % (cfg->key_max - cfg->key_min + 1)) : 0);
        const uint32_t vlen =
            tomb ? klen : (cfg->val_fixed ? cfg->val_fixed : 63u + zipf_sample(thr, (uint32_t)(H(cfg->seed, 2, i) >> 32)));
        const uint64_t entry = 16ull + (tomb ? 0 : klen) + vlen;
        if (size + entry > cfg->max_file_size) {  // rotateDataFile (core/db.go:214-232)
            if (cfg->n_files && cur + 1 >= cfg->n_files) break;
            sizes.push_back(size);
            ++cur;
            size = 0;
        }
        OpDesc o;
        o.dst = size;  // file-relative for now
        o.keyid = keyid;
        o.vlen = vlen;
        o.klen = klen | (tomb ? 0x80000000u : 0u);
        ops.push_back(o);
        op_file.push_back(cur);
        size += entry;
    }
    sizes.push_back(size);
    return GCK_OK;
}

}  // namespace gck

using namespace gck;

extern "C" {

void gck_encode_zipf_table(uint32_t *thr) {
    const auto &t = zipf_thr();
    memcpy(thr, t.data(), t.size() * 4);
}

int gck_encode_corpus(gck_ctx *ctx, const gck_corpus_cfg *cfg, uint32_t *n_files_out, uint64_t *n_ops_out,
                      uint64_t *file_sizes, uint32_t max_files) {
    if (!ctx || !cfg) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    std::vector<OpDesc> ops;
    std::vector<uint32_t> op_file;
    std::vector<uint64_t> sizes;
    int rc = plan(cfg, 0, ops, op_file, sizes);
    if (rc) return rc;
    const uint32_t nf = (uint32_t)sizes.size();
    // walk order = names sorted bytewise (filepath.Walk)
    std::vector<std::string> names(nf);
    for (uint32_t n = 0; n < nf; ++n)
        names[n] = "data_" + std::to_string(n) + "_" + std::to_string((uint32_t)(cfg->ts_base + n)) + ".csk";
    std::vector<uint32_t> order(nf);
    for (uint32_t n = 0; n < nf; ++n) order[n] = n;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return names[a] < names[b]; });
    std::vector<uint32_t> walkpos(nf);
    for (uint32_t w = 0; w < nf; ++w) walkpos[order[w]] = w;
    std::vector<uint64_t> lens(nf);
    std::vector<uint8_t> reset(nf);
    for (uint32_t w = 0; w < nf; ++w) {
        lens[w] = sizes[order[w]];
        reset[w] = w + 1 < nf ? 1 : 0;  // the active file is the lexically last entry
    }
    rc = ctx_layout(c, lens.data(), nf, reset.data());
    if (rc) return rc;
    c->walk_to_creation = order;
    for (size_t i = 0; i < ops.size(); ++i) ops[i].dst += c->f_base[walkpos[op_file[i]]];
    DBuf d_ops;
    if ((rc = d_ops.ensure(ops.size() * sizeof(OpDesc) + 16))) return rc;
    GCK_HIP(hipMemcpy(d_ops.p, ops.data(), ops.size() * sizeof(OpDesc), hipMemcpyHostToDevice));
    if (!ops.empty()) {
        const uint32_t grid = (uint32_t)((ops.size() + 255) / 256);
        k_encode<<<grid, 256, 0, c->stream>>>(c->arena.as<uint8_t>(), d_ops.as<OpDesc>(), ops.size(), cfg->seed,
                                             key_seed_of(cfg), cfg->ts_base, cfg->flip_permille);
        GCK_HIP(hipGetLastError());
    }
    GCK_HIP(hipStreamSynchronize(c->stream));
    d_ops.release();
    if (n_files_out) *n_files_out = nf;
    if (n_ops_out) *n_ops_out = ops.size();
    if (file_sizes)
        for (uint32_t n = 0; n < nf && n < max_files; ++n) file_sizes[n] = sizes[n];
    return GCK_OK;
}

int gck_encode_files(gck_ctx *ctx, const gck_corpus_cfg *cfg, const uint32_t *file_ids, uint32_t n,
                     uint32_t last_is_active, uint64_t *n_ops_out, uint64_t *file_sizes) {
    if (!ctx || !cfg || (n && !file_ids)) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    std::vector<std::vector<OpDesc>> ops(n);
    std::vector<uint64_t> lens(n);
    std::vector<uint8_t> reset(n);
    for (uint32_t k = 0; k < n; ++k) {
        gck_corpus_cfg one = *cfg;
        one.seed = cfg->seed + file_ids[k];
        one.n_files = 1;
        one.n_ops = 0;
        std::vector<uint32_t> op_file;
        std::vector<uint64_t> sizes;
        const int rc = plan(&one, file_ids[k], ops[k], op_file, sizes);
        if (rc) return rc;
        lens[k] = sizes[0];
        reset[k] = (last_is_active && k + 1 == n) ? 0 : 1;
    }
    int rc = ctx_layout(c, lens.data(), n, reset.data());
    if (rc) return rc;
    c->walk_to_creation.assign(file_ids, file_ids + n);
    DBuf d_ops;
    for (uint32_t k = 0; k < n; ++k) {
        for (auto &o : ops[k]) o.dst += c->f_base[k];
        if (ops[k].empty()) continue;
        if ((rc = d_ops.ensure(ops[k].size() * sizeof(OpDesc) + 16))) return rc;
        GCK_HIP(hipMemcpy(d_ops.p, ops[k].data(), ops[k].size() * sizeof(OpDesc), hipMemcpyHostToDevice));
        const uint32_t grid = (uint32_t)((ops[k].size() + 255) / 256);
        k_encode<<<grid, 256, 0, c->stream>>>(c->arena.as<uint8_t>(), d_ops.as<OpDesc>(), ops[k].size(),
                                             cfg->seed + file_ids[k], cfg->key_seed ? cfg->key_seed : cfg->seed + file_ids[k],
                                             cfg->ts_base, cfg->flip_permille);
        GCK_HIP(hipGetLastError());
        GCK_HIP(hipStreamSynchronize(c->stream));  // d_ops is reused by the next file
    }
    d_ops.release();
    uint64_t tot = 0;
    for (uint32_t k = 0; k < n; ++k) {
        tot += ops[k].size();
        if (file_sizes) file_sizes[k] = lens[k];
    }
    if (n_ops_out) *n_ops_out = tot;
    return GCK_OK;
}

int gck_encode_walk_order(gck_ctx *ctx, uint32_t *creation_index, uint32_t n) {
    if (!ctx || !creation_index) return GCK_EINVAL;
    const auto &o = ctx->c.walk_to_creation;
    for (uint32_t i = 0; i < n && i < o.size(); ++i) creation_index[i] = o[i];
    return GCK_OK;
}

}  // extern "C"

// ------------------------------------------------ bulk serializeEntry (f4) ---
// gck_encode_batch: caller records (already in HBM) -> GoCask bytes, back to
// back, as DB.Put / DB.Delete write them (core/db.go:185-212, :245-247,
// serializeEntry :272-284).  Three steps, all on the device:
//   1. record sizes 16 + len(key) + len(value) (a Delete: 16 + len(key)) and
//      their exclusive scan: out_off (k_enc_sizes, k_enc_top, k_enc_add),
//      with the refusals of the host API (an empty key: ErrInvalidKey,
//      core/db.go:186-188 / :294-297; a length past u32; decreasing offsets);
//   2. per wavefront, 64 records: the CRC of each payload (value, or key for a
//      Delete) -- a lane per payload up to 256 B, the whole wavefront in 1 KiB
//      stripes with a ring of stripes in flight for larger ones (gck_crc_wave.h,
//      the machinery of the device Get);
//   3. the wavefront writes its records' output range in 16 B aligned chunks,
//      lane l the chunk at 16 l of each 1 KiB row: a chunk inside one record's
//      key or value is one unaligned 16 B read (two loads + alignbyte) and one
//      aligned 16 B store; a chunk holding header bytes or a record boundary
//      is assembled byte by byte (at most two records meet in 16 B: a record
//      is at least 17 B) and stored whole when it is the group's, else by bytes.
namespace gck {

constexpr uint32_t kEncScanBlock = 1024;

// 1a. sizes, block-local exclusive prefix (into out_off), block sums, refusals
__global__ __launch_bounds__(1024) void k_enc_sizes(const uint64_t *__restrict__ key_off,
                                                   const uint64_t *__restrict__ val_off,
                                                   const uint8_t *__restrict__ tomb, uint64_t n,
                                                   uint64_t *__restrict__ out_off, uint64_t *__restrict__ bsum,
                                                   uint32_t *__restrict__ err) {
    __shared__ uint64_t wsum[16];
    const uint64_t i = (uint64_t)blockIdx.x * kEncScanBlock + threadIdx.x;
    uint64_t sz = 0;
    uint32_t e = 0;
    if (i < n) {
        const uint64_t k0 = key_off[i], k1 = key_off[i + 1], v0 = val_off[i], v1 = val_off[i + 1];
        const bool del = tomb[i] != 0;
        if (k1 < k0 || v1 < v0) e |= 2u;
        const uint64_t kl = k1 - k0, vl = del ? 0 : v1 - v0;
        if (kl == 0) e |= 1u;                                           // ErrInvalidKey
        if (kl > 0xFFFFFFFFull || vl > 0xFFFFFFFFull) e |= 2u;          // u32 header fields
        sz = 16 + kl + vl;
    }
    // exclusive scan over the block: wave scans (u64 in two halves), then the wave totals
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t inc = sz;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    const uint64_t me = __ballot(e != 0);
    if (me && lane == (uint32_t)__builtin_ctzll(me)) atomicOr(err, e);
    __syncthreads();
    uint64_t before = 0;
    for (uint32_t k = 0; k < w; ++k) before += wsum[k];
    if (i < n) out_off[i] = before + inc - sz;
    if (threadIdx.x == blockDim.x - 1) {
        uint64_t tot = 0;
        for (uint32_t k = 0; k < 16; ++k) tot += wsum[k];
        bsum[blockIdx.x] = tot;
    }
}
// 1b. exclusive scan of the block sums (one wavefront); total -> out_off[n]
__global__ void k_enc_top(uint64_t *__restrict__ bsum, uint64_t nb, uint64_t n, uint64_t *__restrict__ out_off,
                          uint64_t *__restrict__ res) {
    const uint32_t lane = threadIdx.x;
    uint64_t run = 0;
    for (uint64_t b0 = 0; b0 < nb; b0 += 64) {
        const uint64_t b = b0 + lane;
        const uint64_t v = b < nb ? bsum[b] : 0;
        uint64_t inc = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(inc, d, 64);
            if (lane >= (uint32_t)d) inc += y;
        }
        if (b < nb) bsum[b] = run + inc - v;
        run += __shfl(inc, 63, 64);
    }
    if (lane == 0) {
        out_off[n] = run;
        res[0] = run;
    }
}
__global__ void k_enc_add(uint64_t *__restrict__ out_off, const uint64_t *__restrict__ bsum, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out_off[i] += bsum[i / kEncScanBlock];
}

// Work units of the encode kernel: unit u = the records whose output starts
// in [u W, (u+1) W), W = 64 KiB (a unit's records may run past its window; a
// record larger than W leaves the units it spans empty).  ufirst[u] = the
// first record starting at or after u W (record r is that for the units in
// (start_{r-1} / W, start_r / W]); ufirst[U] = n.  Units balance the kernel
// by bytes: groups of 64 records differ by orders of magnitude.
constexpr uint64_t kEncUnit = 64 << 10;
constexpr uint32_t kEncThreads = 512;  // k_encode_batch's workgroup (see its launch)
// The unit count from the scan's results on the device (res[0] = the batch's
// bytes, res[1] = refusals): none when the batch is refused, does not fit
// out_cap, or needs more units than the host allotted (units_max: the host
// then runs the call again with enough), so the host launches every kernel
// before it reads anything back.
__device__ __forceinline__ uint64_t enc_units(const uint64_t *res, uint64_t out_cap, uint64_t units_max) {
    const uint64_t total = res[0];
    const uint64_t u = total ? (total - 1) / kEncUnit + 1 : 0;
    return ((uint32_t)res[1] || total > out_cap || u > units_max) ? 0 : u;
}
__global__ void k_enc_units(const uint64_t *__restrict__ out_off, uint64_t n, const uint64_t *__restrict__ res,
                            uint64_t out_cap, uint64_t units_max, uint32_t *__restrict__ ufirst) {
    const uint64_t n_units = enc_units(res, out_cap, units_max);
    if (n_units == 0) return;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= n; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = r < n ? out_off[r] : ~0ull;
        const uint64_t lo = r ? out_off[r - 1] / kEncUnit + 1 : 0;
        const uint64_t hi = r < n ? s / kEncUnit : n_units;  // inclusive
        for (uint64_t u = lo; u <= hi && u <= n_units; ++u) ufirst[u] = (uint32_t)r;
    }
}

// The 16 bytes at src (any alignment): two dword-aligned loads, a byte shift.
// Reads the dwords holding [src, src + 16) only: the second load is the dword
// after the first 16 B when src is unaligned (it holds bytes of the window),
// else a dword inside them (alignbyte by 0 ignores it).  With a 4-byte aligned
// blob base nothing outside the blob's dwords is read (gck_encode_batch checks
// the alignment).
__device__ __forceinline__ uint4 load16u(const uint8_t *src) {
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3);
    const uint8_t *a = src - sh;
    const u32x4_a4 x = *reinterpret_cast<const u32x4_a4 *>(a);
    const uint32_t y = *reinterpret_cast<const uint32_t *>(a + (sh ? 16 : 12));
    return make_uint4(__builtin_amdgcn_alignbyte(x.y, x.x, sh), __builtin_amdgcn_alignbyte(x.z, x.y, sh),
                      __builtin_amdgcn_alignbyte(x.w, x.z, sh), __builtin_amdgcn_alignbyte(y, x.w, sh));
}


__device__ __forceinline__ CrcTabs &enc_tabs() {
    __shared__ CrcTabs t;
    return t;
}
// Per group of 64 records: the payload CRCs (the LDS tables; one workgroup
// of kEncThreads per CU), a payload larger than kLaneMax copied to the output from the
// stripe registers of its CRC (gck_crc_wave.h fold_stripe<true>: no second
// read), then a lane per record writes its header (the CRC from a register),
// key and the rest of a small payload as 16 B pieces.  Round 3's copy pass
// over 1 KiB output rows re-read the payloads from L2 and assembled the rows
// holding record boundaries byte by byte: 1.22 ms per GB against 0.68 now
// (DESIGN.md §10e).
__global__ __launch_bounds__(kEncThreads) void k_encode_batch(const uint8_t *__restrict__ keys,
                                                       const uint64_t *__restrict__ key_off,
                                                       const uint8_t *__restrict__ vals,
                                                       const uint64_t *__restrict__ val_off,
                                                       const uint32_t *__restrict__ ts,
                                                       const uint8_t *__restrict__ tomb, uint64_t n,
                                                       const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
                                                       const uint32_t *__restrict__ ufirst,
                                                       const uint64_t *__restrict__ res, uint64_t out_cap,
                                                       uint64_t units_max, uint32_t *__restrict__ queue) {
    const uint64_t n_units = enc_units(res, out_cap, units_max);
    if (n_units == 0) return;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t lb0 = 0, lb1 = 0, kl_shift = 0;
    CrcTabs *T = &enc_tabs();
    const uint64_t key_total = key_off[n], val_total = val_off[n];  // the blobs' sizes
    // the slicing tables, built here (no context): T0..T3 into Zs, expanded
    // into the conflict-free image, then Zs itself
    {
        uint32_t *t4 = &T->Zs[0][0];
        for (uint32_t v = threadIdx.x; v < 256; v += blockDim.x) {
            uint32_t c = v;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
            t4[v] = c;
        }
        __syncthreads();
        for (uint32_t v = threadIdx.x; v < 256; v += blockDim.x) {
            uint32_t c = t4[v];
            for (int k = 1; k < 4; ++k) {
                c = (c >> 8) ^ t4[c & 0xFF];
                t4[k * 256 + v] = c;
            }
        }
        __syncthreads();
        fill_slice_lds(T->S, t4);
        __syncthreads();
        fill_zs(*T);
        __syncthreads();
        slice_bases(lane, lb0, lb1);
        kl_shift = xpow8n(16ull * (63 - lane));
    }
    // units from an atomic queue, each as groups of up to 64 records
    for (;;) {
        uint32_t u = 0;
        if (lane == 0) u = atomicAdd(queue, 1u);
        u = (uint32_t)__builtin_amdgcn_readfirstlane((int)u);
        if (u >= n_units) break;
        const uint64_t ua = ufirst[u], ub = ufirst[u + 1];
    for (uint64_t g0 = ua; g0 < ub; g0 += 64) {
        const uint64_t mine = g0 + lane;
        const uint32_t cnt = (uint32_t)min<uint64_t>(64, ub - g0);
        const bool have = mine < g0 + cnt;
        const uint64_t ko = have ? key_off[mine] : 0, kl = have ? key_off[mine + 1] - ko : 0;
        const bool del = have && tomb[mine] != 0;
        const uint64_t vo = have ? val_off[mine] : 0, vl = have && !del ? val_off[mine + 1] - vo : 0;
        const uint32_t t = have ? ts[mine] : 0u;
        const uint64_t oo = have ? out_off[mine] : 0;
        // 2. CRCs: a lane per small payload (and per payload at its blob's
        // first 16 bytes: the stripe reads may reach 15 bytes before it),
        // the wavefront for the rest
        const uint64_t po = del ? ko : vo;
        const uint32_t L = (uint32_t)(del ? kl : vl);
        const bool small = have && (L <= kLaneMax || po < 16);
        uint32_t crc = 0;
        // (its whole 16 B pieces copied to the output from the same
        // registers).  16 B loads where the blob holds 16 bytes past the
        // payload (wide: the loads may reach 15 bytes past its last byte),
        // dword loads for the rest (the blob's last payloads)
        const bool wide = small && po + L + 16 <= (del ? key_total : val_total);
        if (__ballot(wide)) {
            const uint32_t c = lane_crc<true, true, 32>((del ? keys : vals) + po, L, wide, *T, lb0, lb1,
                                                    out + oo + 16 + (del ? 0 : kl));
            if (wide) crc = c;
        }
        if (__ballot(small && !wide)) {
            const uint32_t c = lane_crc<false, true>((del ? keys : vals) + po, L, small && !wide, *T, lb0, lb1,
                                                     out + oo + 16 + (del ? 0 : kl));
            if (small && !wide) crc = c;
        }
        const uint64_t todo = __ballot(have && !small);
        if (todo) {
            // the payload's copy from the stripe registers: out + ps
            const uint64_t ps = oo + 16 + (del ? 0 : kl);
            const uint32_t c = wave_crcs<false, true>(
                todo, [&](int it) { return (lane_u32(del, it) ? keys : vals) + lane_u64(po, it); }, L, *T, lb0,
                lb1, [&](uint32_t A) { return lanes_combine_gmul(kl_shift, A); },
                [&](int it) { return out + lane_u64(ps, it); });
            if ((todo >> lane) & 1) crc = c;
        }
        const uint32_t h1 = t, h2 = del ? 0u : (uint32_t)kl, h3 = (uint32_t)(del ? kl : vl);
        // 3. the rest of the group's output, a lane per record, as 16 B
        // pieces at any alignment inside the record: a payload the wave path
        // copied (above) needs only its first 16 bytes, a small one (whose
        // whole pieces lane_crc stored) its last L % 16.  A piece that ends at the end of a region and starts
        // before it (a key or value shorter than 16 B) carries wrong bytes in
        // front; the lane writes its pieces from the record's end back to its
        // header, so its later stores overwrite them (one thread's stores to
        // one address land in program order).  Bytes written twice are the
        // same bytes.
        if (have) {
            const uint64_t vsx = oo + 16 + kl, vex = vsx + vl;  // the value's output range
            if (vl >= 16) {
                if (!small)
                    store16u(out + vsx, load16u(vals + vo));
                else if (vl & 15)
                    store16u(out + vex - 16, load16u(vals + vo + vl - 16));
            } else if (vl && vo + vl >= 16) {  // reaches back into the key / header
                store16u(out + vex - 16, load16u(vals + vo + vl - 16));
            } else {
                for (uint32_t i = 0; i < (uint32_t)vl; ++i) out[vsx + i] = vals[vo + i];  // (the blob's first bytes)
            }
            const uint64_t ks = oo + 16;
            if (kl & 15) {
                if (ko + kl >= 16) {
                    store16u(out + ks + kl - 16, load16u(keys + ko + kl - 16));
                } else {
                    for (uint32_t i = 0; i < (uint32_t)kl; ++i) out[ks + i] = keys[ko + i];
                }
            }
            for (uint64_t i = 0; i + 16 <= kl; i += 16) store16u(out + ks + i, load16u(keys + ko + i));
            store16u(out + oo, make_uint4(crc, h1, h2, h3));
        }
    }
    }
}

}  // namespace gck

extern "C" int gck_encode_batch(const uint8_t *keys, const uint64_t *key_off, const uint8_t *vals,
                                const uint64_t *val_off, const uint32_t *ts, const uint8_t *tomb, uint64_t n,
                                uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *total,
                                void *stream) {
    if (!key_off || !val_off || !out_off || !total || (n && (!keys || !out || !ts || !tomb))) return GCK_EINVAL;
    // the kernels read whole dwords of the key / value blobs from their base
    if ((reinterpret_cast<uintptr_t>(keys) | reinterpret_cast<uintptr_t>(vals)) & 3) return GCK_EINVAL;
    int ndev = 0, dev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || hipGetDevice(&dev) != hipSuccess) return GCK_EDEVICE;
    hipStream_t s = (hipStream_t)stream;
    *total = 0;
    int n_cu = 0;
    GCK_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    // one scratch block: block sums, results (total, refusals), the unit
    // queue, ufirst for as many units as out_cap holds.  Every kernel is
    // launched before the one readback (the sizes' verdict is applied on the
    // device, enc_units): one host round trip per call instead of two.
    size_t dev_mem = 0;  // (an output larger than the device's memory: a second pass, below)
    GCK_HIP(hipDeviceTotalMem(&dev_mem, dev));
    const uint64_t nb = (n + kEncScanBlock - 1) / kEncScanBlock;
    uint64_t units_max = (std::min<uint64_t>(out_cap, dev_mem) + kEncUnit - 1) / kEncUnit;
    for (;;) {
        units_max = std::max<uint64_t>(units_max, 1);
        void *tmp = nullptr;
        GCK_HIP(hipMallocAsync(&tmp, (nb + 1) * 8 + 24 + (units_max + 1) * 4, s));
        uint64_t *bsum = static_cast<uint64_t *>(tmp), *res = bsum + nb + 1;
        uint32_t *queue = reinterpret_cast<uint32_t *>(res + 2), *ufirst = queue + 2;
        GCK_HIP(hipMemsetAsync(res, 0, 24, s));
        // 1. sizes and offsets on the device
        if (n) k_enc_sizes<<<(uint32_t)nb, kEncScanBlock, 0, s>>>(key_off, val_off, tomb, n, out_off, bsum,
                                                                  reinterpret_cast<uint32_t *>(res + 1));
        k_enc_top<<<1, 64, 0, s>>>(bsum, nb, n, out_off, res);
        if (n) {
            k_enc_add<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(out_off, bsum, n);
            // units of 64 KiB of output: the last record starts before the total
            // (units past its start stay empty, k_enc_units)
            k_enc_units<<<(uint32_t)std::min<uint64_t>((n + 256) / 256, 4096), 256, 0, s>>>(out_off, n, res, out_cap,
                                                                                           units_max, ufirst);
            // one workgroup per CU (the CRC tables take 152 KiB of LDS) of 8
            // wavefronts: 0.68-0.69 ms per GB against 0.71-0.72 with 16 (the
            // memory system, not latency, is what more wavefronts add to), 0.69
            // with 12, 0.76 with 6, 0.95 with 4 (profiles/r4zu, r4zv)
            const uint32_t grid = (uint32_t)std::min<uint64_t>((units_max + 7) / 8, (uint64_t)n_cu);
            k_encode_batch<<<grid, kEncThreads, 0, s>>>(keys, key_off, vals, val_off, ts, tomb, n, out_off, out, ufirst,
                                                  res, out_cap, units_max, queue);
            GCK_HIP(hipGetLastError());
        }
        uint64_t h[2] = {0, 0};
        GCK_HIP(hipMemcpyAsync(h, res, 16, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipStreamSynchronize(s));
        (void)hipFreeAsync(tmp, s);
        const uint32_t err = (uint32_t)h[1];
        if (err & 1u) return GCK_EINVALID_KEY;  // Put / Delete of an empty key (core/db.go:186, :294)
        if (err & 2u) return GCK_EINVAL;        // decreasing offsets, or u32 header fields overflow
        *total = h[0];
        if (*total > out_cap) return GCK_EINVAL;  // *total says how much is needed (nothing was written)
        const uint64_t need = *total ? (*total - 1) / kEncUnit + 1 : 0;
        if (need <= units_max) break;
        units_max = need;  // an output past the device's memory (mapped host memory): again, with room
    }
    return GCK_OK;
}

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

namespace gck {

constexpr uint32_t kZipfN = 65473;

static std::vector<uint32_t> &zipf_thr() {
    static std::vector<uint32_t> thr;
    if (thr.empty()) {
        std::vector<double> cum(kZipfN);
        double acc = 0.0;
        for (uint32_t r = 1; r <= kZipfN; ++r) {
            acc += std::pow((double)r, -1.1);
            cum[r - 1] = acc;
        }
        thr.resize(kZipfN - 1);
        for (uint32_t k = 0; k + 1 < kZipfN; ++k) {
            const double v = std::floor(cum[k] / acc * 4294967296.0);
            thr[k] = v >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)v;
        }
    }
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
                                                uint64_t n_ops, uint64_t seed, uint32_t ts_base,
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
    const uint64_t w0 = mix64(o.keyid ^ H(seed, 7, 0));
    uint32_t kc = 0xFFFFFFFFu;
    for (uint32_t j = 0; j < klen; ++j) {
        const uint64_t w = j < 8 ? w0 : H(seed, 8, o.keyid * 64 + j / 8);
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
static int plan(const gck_corpus_cfg *cfg, std::vector<OpDesc> &ops, std::vector<uint32_t> &op_file,
                std::vector<uint64_t> &sizes) {
    if (cfg->key_min < 8 || cfg->key_max > 512 || cfg->key_max < cfg->key_min) return GCK_EINVAL;
    if (!cfg->n_ops && !cfg->n_files) return GCK_EINVAL;
    if (!cfg->val_fixed && cfg->max_file_size == 0) return GCK_EINVAL;
    if (cfg->val_fixed >= (1u << 23)) return GCK_EINVAL;
    const auto &thr = zipf_thr();
    uint32_t cur = 0;
    uint64_t size = 0;
    sizes.clear();
    for (uint64_t i = 0;; ++i) {
        if (cfg->n_ops && i >= cfg->n_ops) break;
        const bool tomb = cfg->tomb_permille && (H(cfg->seed, 3, i) % 1000u) < cfg->tomb_permille;
        const uint64_t keyid = cfg->key_universe ? H(cfg->seed, 1, i) % cfg->key_universe : i;
        const uint32_t klen =
            cfg->key_min +
            (cfg->key_max > cfg->key_min ? (uint32_t)(H(cfg->seed, 6, keyid) % (cfg->key_max - cfg->key_min + 1)) : 0);
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
    int rc = plan(cfg, ops, op_file, sizes);
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
                                             cfg->ts_base, cfg->flip_permille);
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
        const int rc = plan(&one, ops[k], op_file, sizes);
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
                                             cfg->seed + file_ids[k], cfg->ts_base, cfg->flip_permille);
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
// serializeEntry :272-284).  One wavefront per record: the lanes copy key and
// value with strided byte stores and CRC the payload in 64 contiguous
// segments, combined through Z_n (gck_math.h):
//   F(0, V) = XOR_l Z_{|V| - end_l}(F(0, seg_l)),  crc = ~(F(0,V) ^ Z_|V|(~0)).
namespace gck {

__global__ __launch_bounds__(256) void k_encode_batch(const uint8_t *__restrict__ keys,
                                                      const uint64_t *__restrict__ key_off,
                                                      const uint8_t *__restrict__ vals,
                                                      const uint64_t *__restrict__ val_off,
                                                      const uint32_t *__restrict__ ts,
                                                      const uint8_t *__restrict__ tomb, uint64_t n,
                                                      const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out) {
    __shared__ uint32_t T[256];
    for (uint32_t v = threadIdx.x; v < 256; v += blockDim.x) {
        uint32_t c = v;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
        T[v] = c;
    }
    __shared__ uint32_t X8[64];  // x^(8 * 2^k) mod P: powers by set bits, no squarings
    if (threadIdx.x == 0) {
        uint32_t x = kX0 >> 8;
        for (int k = 0; k < 64; ++k) {
            X8[k] = x;
            x = multmodp(x, x);
        }
    }
    __syncthreads();
    auto zpow = [&](uint64_t m) {  // x^(8m) mod P
        uint32_t r = kX0;
        for (; m; m &= m - 1) r = multmodp(X8[__builtin_ctzll(m)], r);
        return r;
    };
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    // records in groups of 64 per wavefront: payloads up to kLaneMax bytes (1 KiB: A/B of 512..4096, tools/xp_lane_max.sh) are
    // encoded by one lane each (a serial CRC, no GF(2) combine), larger ones by
    // the whole wavefront, one after another
#ifndef GCK_LANE_MAX
#define GCK_LANE_MAX 1024
#endif
    constexpr uint64_t kLaneMax = GCK_LANE_MAX;
    for (uint64_t g = wave * 64; g < n; g += n_waves * 64) {
        const uint64_t li = g + lane;
        bool big = false;
        if (li < n) {
            const bool del = tomb[li] != 0;
            const uint8_t *key = keys + key_off[li];
            const uint64_t kl = key_off[li + 1] - key_off[li];
            const uint8_t *val = vals + val_off[li];
            const uint64_t vl = del ? 0 : val_off[li + 1] - val_off[li];
            big = (del ? kl : vl) > kLaneMax;
            if (!big) {
                uint8_t *dst = out + out_off[li];
                uint32_t c = 0xFFFFFFFFu;
                // bytes of src to d, eight aligned dwords in flight; CRC'd when crc
                auto put = [&](const uint8_t *src, uint8_t *d, uint64_t len, bool crc) {
                    auto one = [&](uint64_t j, uint8_t x) {
                        d[j] = x;
                        if (crc) c = T[(c ^ x) & 0xff] ^ (c >> 8);
                    };
                    uint64_t j = 0;
                    const uint64_t al = min(len, (uint64_t)((4u - ((uintptr_t)src & 3u)) & 3u));
                    for (; j < al; ++j) one(j, src[j]);
                    const uint32_t *pw = reinterpret_cast<const uint32_t *>(src + j);
                    const uint64_t nw = (len - j) / 4;
                    uint64_t q = 0;
                    for (; q + 8 <= nw; q += 8) {
                        uint32_t v[8];
#pragma unroll
                        for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(pw + q + k);
#pragma unroll
                        for (int k = 0; k < 8; ++k)
#pragma unroll
                            for (int b = 0; b < 4; ++b) one(j + 4 * (q + k) + b, (uint8_t)(v[k] >> (8 * b)));
                    }
                    for (; q < nw; ++q) {
                        const uint32_t w = pw[q];
#pragma unroll
                        for (int b = 0; b < 4; ++b) one(j + 4 * q + b, (uint8_t)(w >> (8 * b)));
                    }
                    for (j += 4 * nw; j < len; ++j) one(j, src[j]);
                };
                put(key, dst + 16, kl, del);
                put(val, dst + 16 + kl, vl, !del);
                const uint32_t hv[4] = {~c, ts[li], del ? 0u : (uint32_t)kl, (uint32_t)(del ? kl : vl)};
#pragma unroll
                for (int k = 0; k < 16; ++k) dst[k] = (uint8_t)(hv[k / 4] >> (8 * (k % 4)));
            }
        }
        uint64_t bigs = __ballot(big);
        while (bigs) {
        const uint64_t i = g + (uint64_t)__builtin_ctzll(bigs);
        bigs &= bigs - 1;
        const bool del = tomb[i] != 0;
        const uint8_t *key = keys + key_off[i];
        const uint64_t kl = key_off[i + 1] - key_off[i];
        const uint8_t *val = vals + val_off[i];
        const uint64_t vl = del ? 0 : val_off[i + 1] - val_off[i];
        uint8_t *dst = out + out_off[i];
        // coalesced byte copies, eight loads in flight per lane before the stores
        auto copy = [&](const uint8_t *src, uint8_t *d, uint64_t len) {
            uint64_t j = lane;
            for (; j + 7 * 64 < len; j += 8 * 64) {
                uint8_t v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(src + j + 64 * k);
#pragma unroll
                for (int k = 0; k < 8; ++k) d[j + 64 * k] = v[k];
            }
            for (; j < len; j += 64) d[j] = src[j];
        };
        copy(key, dst + 16, kl);
        copy(val, dst + 16 + kl, vl);
        // the CRC payload: the value (Put) or the key (Delete)
        const uint8_t *pl = del ? key : val;
        const uint64_t len = del ? kl : vl;
        const uint64_t seg = (len + 63) / 64, b = min(len, lane * seg), e = min(len, b + seg);
        // the lane's segment: head bytes up to a 4 B boundary, aligned dwords
        // eight at a time (independent loads in flight), tail bytes
        uint32_t c = 0;
        auto byte = [&](uint8_t x) { c = T[(c ^ x) & 0xff] ^ (c >> 8); };
        auto word = [&](uint32_t w) {
#pragma unroll
            for (int k = 0; k < 4; ++k) byte((uint8_t)(w >> (8 * k)));
        };
        uint64_t j = b;
        const uint64_t al = min(e, b + ((4u - ((uintptr_t)(pl + b) & 3u)) & 3u));
        for (; j < al; ++j) byte(pl[j]);
        const uint32_t *pw = reinterpret_cast<const uint32_t *>(pl + j);
        const uint64_t nw = (e - j) / 4;
        uint64_t q = 0;
        for (; q + 8 <= nw; q += 8) {
            uint32_t v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(pw + q + k);
#pragma unroll
            for (int k = 0; k < 8; ++k) word(v[k]);
        }
        for (; q < nw; ++q) word(pw[q]);
        for (j += 4 * nw; j < e; ++j) byte(pl[j]);
        uint32_t f = c ? multmodp(zpow(len - e), c) : 0u;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) f ^= (uint32_t)__shfl_xor((int)f, m, 64);
        const uint32_t crc = ~(f ^ multmodp(zpow(len), 0xFFFFFFFFu));
        const uint32_t hv[4] = {crc, ts[i], del ? 0u : (uint32_t)kl, (uint32_t)(del ? kl : vl)};
        if (lane < 16) dst[lane] = (uint8_t)(hv[lane / 4] >> (8 * (lane % 4)));
        }
    }
}

}  // namespace gck

extern "C" int gck_encode_batch(const uint8_t *keys, const uint64_t *key_off, const uint8_t *vals,
                                const uint64_t *val_off, const uint32_t *ts, const uint8_t *tomb, uint64_t n,
                                uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *total,
                                void *stream) {
    if (!key_off || !val_off || !out_off || !total || (n && (!keys || !out || !ts || !tomb))) return GCK_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GCK_EDEVICE;
    hipStream_t s = (hipStream_t)stream;
    // record offsets: a sequential sum over the sizes (17 B per record crosses
    // PCIe twice; the bytes themselves never leave the device)
    std::vector<uint64_t> ko(n + 1), vo(n + 1), off(n + 1);
    std::vector<uint8_t> tb(n);
    GCK_HIP(hipMemcpyAsync(ko.data(), key_off, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipMemcpyAsync(vo.data(), val_off, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    if (n) GCK_HIP(hipMemcpyAsync(tb.data(), tomb, n, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    off[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (ko[i + 1] < ko[i] || vo[i + 1] < vo[i]) return GCK_EINVAL;
        const uint64_t kl = ko[i + 1] - ko[i], vl = tb[i] ? 0 : vo[i + 1] - vo[i];
        if (kl == 0) return GCK_EINVALID_KEY;  // Put / Delete of an empty key (core/db.go:186, :294)
        if (kl > 0xFFFFFFFFull || vl > 0xFFFFFFFFull) return GCK_EINVAL;  // u32 header fields
        off[i + 1] = off[i] + 16 + kl + vl;
    }
    *total = off[n];
    if (*total > out_cap) return GCK_EINVAL;  // *total says how much is needed
    GCK_HIP(hipMemcpyAsync(out_off, off.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
    if (n) {
        const uint64_t waves = std::min<uint64_t>((n + 63) / 64, 256ull * 64);
        k_encode_batch<<<(uint32_t)((waves + 3) / 4), 256, 0, s>>>(keys, key_off, vals, val_off, ts, tomb, n,
                                                                   out_off, out);
        GCK_HIP(hipGetLastError());
    }
    GCK_HIP(hipStreamSynchronize(s));
    return GCK_OK;
}

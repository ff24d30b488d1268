/*
 * shim_test.c — TEST PROGRAM.  Does in C exactly what the cgo shim of
 * INTEGRATION.md §2 does inside core.NewDB, so the calling pattern a Go
 * maintainer would ship is exercised against the real library:
 *
 *   1. walk the db directory like Disk.Walk (internal/fs/disk.go:122-145):
 *      filepath.Walk order (names sorted bytewise, recursive, Lstat), only
 *      *.csk; each file is opened read-only, and INSIDE the walk callback,
 *      while it is open, stat'ed, mmap'ed read-only and page-locked
 *      (gck_host_register) -- Disk.Walk closes it when the callback returns
 *      (disk.go:143), the mapping stays valid;
 *   2. reset_after = Name() != activeFile.Name() (core/db.go:117);
 *   3. no .csk file at all: nothing to replay, an empty keydir (the shim
 *      must not index files[0]);
 *   4. gck_replay through include/gocask_hip.h;
 *   5. apply the records in walk order to a map (keyDir.set / unset,
 *      core/keydir.go:22-49) and lastOffset = final_last_offset.
 *
 * Usage: shim_test <db dir> [active Name()]   (default: Disk.Open's choice,
 * the lexically last directory entry without its extension).
 * Prints "status <rc> last_offset <n> keys <n>" then one line per live key:
 * "<key hex> <crc> <ts> <value_pos> <value_size> <file Name()>", sorted.
 * SHIM_TIME=1: time the Open as the shim pays it (walk + stat + mmap +
 * gck_host_register inside the callback, gck_replay, gck_result_free,
 * unregister + munmap) and print one JSON line instead of the keys.
 * SHIM_MULTI=1: gck_replay_multi on device 0 (the live keydir comes back).
 * SHIM_PIN=0: map the files but do not register them (the library stages the
 * pageable mappings through its own page-locked buffers).
 * SHIM_PATHS=1: gck_replay_paths (with SHIM_MULTI=1 gck_replay_multi_paths)
 * -- the library opens and reads the files itself (the shim maps them only
 * to print keys, never when timing).
 * SHIM_LIVE=1: GCK_OPT_LIVE -- the single-GPU call returns the live keydir
 * (the device keydir, merged over the file groups) instead of every record.
 * Timing mode also fills the keydir map as the Go shim does after the call
 * (map_fill.cpp: a std::unordered_map<std::string, entry>, the Go map's
 * proxy; every record set / unset in walk order, or one insert per live
 * key), with the key bytes from GCK_OPT_KEYS, and includes it in open_ms.
 */
#define _GNU_SOURCE
#include <dirent.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "gocask_hip.h"

double shim_map_fill(const gck_rec *recs, uint64_t n, const uint8_t *keys, int live, uint64_t *n_live);

typedef struct {
    char name[256]; /* DiskFile.Name(): base name without the extension */
    char *path;
    const uint8_t *map;
    uint64_t len;
    int pinned;
} mapped;

static mapped *g_files;
static size_t g_n, g_cap;
static int g_pin = 1, g_map = 1;

static int cmp_str(const void *a, const void *b) { return strcmp(*(char *const *)a, *(char *const *)b); }

static const char *ext_of(const char *p) {
    const char *d = strrchr(p, '.'), *s = strrchr(p, '/');
    return d && (!s || d > s) ? d : "";
}

/* The Walk callback: the file is open here and only here. */
static int on_file(const char *path) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) return -1;
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        return -1;
    }
    if (g_n == g_cap) {
        g_cap = g_cap ? 2 * g_cap : 16;
        g_files = realloc(g_files, g_cap * sizeof(mapped));
    }
    mapped *m = &g_files[g_n++];
    memset(m, 0, sizeof *m);
    const char *b = strrchr(path, '/');
    b = b ? b + 1 : path;
    snprintf(m->name, sizeof m->name, "%.*s", (int)(ext_of(b) - b), b);
    m->len = (uint64_t)st.st_size;
    m->path = strdup(path);
    if (m->len && g_map) {
        void *a = mmap(NULL, m->len, PROT_READ, MAP_SHARED, fd, 0);
        if (a == MAP_FAILED) {
            close(fd);
            return -1;
        }
        m->map = a;
        /* pinning is an optimisation only */
        m->pinned = g_pin && gck_host_register(m->map, m->len) == GCK_OK;
    }
    close(fd); /* Disk.Walk: return file.Close() */
    return 0;
}

static int walk(const char *path) { /* filepath.Walk with Disk.Walk's filter */
    struct stat st;
    if (lstat(path, &st) != 0) return -1;
    if (!S_ISDIR(st.st_mode)) return strcmp(ext_of(path), ".csk") == 0 ? on_file(path) : 0;
    DIR *d = opendir(path);
    if (!d) return -1;
    char **names = NULL;
    size_t n = 0, cap = 0;
    for (struct dirent *e; (e = readdir(d));) {
        if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
        if (n == cap) names = realloc(names, (cap = cap ? 2 * cap : 16) * sizeof(char *));
        names[n++] = strdup(e->d_name);
    }
    closedir(d);
    qsort(names, n, sizeof(char *), cmp_str);
    int rc = 0;
    for (size_t i = 0; i < n; ++i) {
        char *p = NULL;
        if (!rc && asprintf(&p, "%s/%s", path, names[i]) > 0) rc = walk(p);
        free(p);
        free(names[i]);
    }
    free(names);
    return rc;
}

typedef struct {
    const uint8_t *key;
    uint32_t klen;
    gck_rec rec;
    int live;
} kd_entry;

static int cmp_kd(const void *a, const void *b) {
    const kd_entry *x = a, *y = b;
    const uint32_t n = x->klen < y->klen ? x->klen : y->klen;
    const int c = memcmp(x->key, y->key, n);
    return c ? c : (x->klen > y->klen) - (x->klen < y->klen);
}

static void release_files(void) {
    for (size_t i = 0; i < g_n; ++i) {
        if (g_files[i].pinned) gck_host_unregister(g_files[i].map);
        if (g_files[i].map) munmap((void *)g_files[i].map, g_files[i].len);
        free(g_files[i].path);
    }
}

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

int main(int argc, char **argv) {
    const int timing = getenv("SHIM_TIME") && atoi(getenv("SHIM_TIME"));
    const int multi = getenv("SHIM_MULTI") && atoi(getenv("SHIM_MULTI"));
    const int by_path = getenv("SHIM_PATHS") && atoi(getenv("SHIM_PATHS"));
    const int live_mode = getenv("SHIM_LIVE") && atoi(getenv("SHIM_LIVE"));
    if (getenv("SHIM_PIN")) g_pin = atoi(getenv("SHIM_PIN"));
    if (by_path) g_pin = 0;
    if (by_path && timing) g_map = 0;
    if (argc < 2) {
        fprintf(stderr, "usage: %s <db dir> [active name]\n", argv[0]);
        return 2;
    }
    char active[256] = "";
    if (argc > 2) {
        snprintf(active, sizeof active, "%s", argv[2]);
    } else { /* Disk.Open: the lexically last entry of any kind */
        struct dirent **ents;
        int n = scandir(argv[1], &ents, NULL, alphasort);
        for (int i = 0; i < n; ++i) {
            if (strcmp(ents[i]->d_name, ".") && strcmp(ents[i]->d_name, "..")) {
                const char *e = ext_of(ents[i]->d_name);
                snprintf(active, sizeof active, "%.*s", (int)(e - ents[i]->d_name), ents[i]->d_name);
            }
            free(ents[i]);
        }
        if (n >= 0) free(ents);
    }
    const double t0 = now_ms();
    if (walk(argv[1]) != 0) {
        fprintf(stderr, "walk failed\n");
        return 3;
    }
    const double t1 = now_ms();
    int rc = GCK_OK;
    gck_result res;
    memset(&res, 0, sizeof res);
    gck_opts opts;
    memset(&opts, 0, sizeof opts);
    opts.flags = (live_mode ? GCK_OPT_LIVE : 0u) | (timing ? GCK_OPT_KEYS : 0u);
    if (g_n) { /* zero files: no replay, no files[0] */
        gck_file *gf = calloc(g_n, sizeof(gck_file));
        for (size_t i = 0; i < g_n; ++i) {
            gf[i].data = g_files[i].map;
            gf[i].len = g_files[i].len;
            gf[i].reset_after = strcmp(g_files[i].name, active) != 0;
        }
        if (by_path) {
            gck_path *gp = calloc(g_n, sizeof(gck_path));
            for (size_t i = 0; i < g_n; ++i) {
                gp[i].path = g_files[i].path;
                gp[i].reset_after = gf[i].reset_after;
            }
            if (multi) {
                const int32_t dev0 = 0;
                rc = gck_replay_multi_paths(gp, (uint32_t)g_n, &dev0, 1, &opts, &res);
            } else {
                rc = gck_replay_paths(gp, (uint32_t)g_n, &opts, &res);
            }
            free(gp);
        } else if (multi) {
            const int32_t dev0 = 0;
            rc = gck_replay_multi(gf, (uint32_t)g_n, &dev0, 1, &opts, &res);
        } else {
            rc = gck_replay(gf, (uint32_t)g_n, &opts, &res);
        }
        free(gf);
        if (rc != GCK_OK && rc != GCK_EUNEXPECTED_EOF) {
            fprintf(stderr, "gck_replay: %d %s\n", rc, gck_last_error());
            return 4;
        }
    }
    const double t2 = now_ms();
    if (timing) {
        uint64_t bytes = 0;
        for (size_t i = 0; i < g_n; ++i) bytes += g_files[i].len;
        const uint64_t n = res.n, fail = res.n_crc_fail;
        const uint32_t last = res.final_last_offset, groups = res.n_groups, resident = res.n_resident;
        /* the Go shim's keydir fill (records set / unset in walk order, or
         * one insert per live entry), keys from GCK_OPT_KEYS */
        uint64_t n_map = 0;
        const double fill_ms = n ? shim_map_fill(res.recs, n, res.keys, live_mode || multi, &n_map) : 0.0;
        const double t2b = now_ms();
        if (g_n) gck_result_free(&res);
        const double t3 = now_ms();
        release_files();
        const double t4 = now_ms();
        printf("{\"files\": %zu, \"bytes\": %llu, \"status\": %d, \"records\": %llu, \"crc_rejects\": %llu, "
               "\"last_offset\": %u, \"groups\": %u, \"resident\": %u, \"walk_mmap_register_ms\": %.2f, "
               "\"replay_ms\": %.2f, \"map_fill_ms\": %.2f, \"map_entries\": %llu, \"free_ms\": %.2f, "
               "\"unregister_unmap_ms\": %.2f, \"open_ms\": %.2f, "
               "\"open_gib_s\": %.3f, \"multi\": %d, \"live\": %d, \"mode\": \"%s\"}\n",
               g_n, (unsigned long long)bytes, rc, (unsigned long long)n, (unsigned long long)fail, last, groups,
               resident, t1 - t0, t2 - t1, fill_ms, (unsigned long long)n_map, t3 - t2b, t4 - t3, t4 - t0,
               bytes / ((t4 - t0) * 1e-3) / (1 << 30), multi, live_mode, by_path ? "paths" : g_pin ? "pinned" : "pageable");
        (void)fill_ms;
        free(g_files);
        return 0;
    }
    /* keyDir.set / unset in walk order: a sorted array, last writer wins */
    kd_entry *kd = calloc(res.n ? res.n : 1, sizeof(kd_entry));
    size_t nk = 0;
    for (uint64_t i = 0; i < res.n; ++i) {
        const gck_rec *r = &res.recs[i];
        kd[nk].key = g_files[r->file].map + r->rec_off + 16;
        kd[nk].klen = r->key_len;
        kd[nk].rec = *r;
        kd[nk].live = !(r->flags & GCK_F_TOMBSTONE);
        ++nk;
    }
    /* stable: equal keys keep walk order, the last one wins */
    for (size_t i = 1; i < nk; ++i) { /* insertion sort by key (test sizes) */
        kd_entry t = kd[i];
        size_t j = i;
        while (j > 0 && cmp_kd(&kd[j - 1], &t) > 0) {
            kd[j] = kd[j - 1];
            --j;
        }
        kd[j] = t;
    }
    size_t live = 0;
    for (size_t i = 0; i < nk; ++i)
        if ((i + 1 == nk || cmp_kd(&kd[i], &kd[i + 1]) != 0) && kd[i].live) ++live;
    printf("status %d last_offset %u keys %zu\n", rc, res.final_last_offset, live);
    for (size_t i = 0; i < nk; ++i) {
        if (!((i + 1 == nk || cmp_kd(&kd[i], &kd[i + 1]) != 0) && kd[i].live)) continue;
        for (uint32_t b = 0; b < kd[i].klen; ++b) printf("%02x", kd[i].key[b]);
        const gck_rec *r = &kd[i].rec;
        printf(" %u %u %u %u %s\n", r->crc, r->ts, r->value_pos, r->value_size, g_files[r->file].name);
    }
    free(kd);
    if (g_n) gck_result_free(&res);
    release_files();
    free(g_files);
    return 0;
}

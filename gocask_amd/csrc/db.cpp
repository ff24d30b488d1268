// db.cpp — host-side mirror of the reference's embedding surface around replay.
//
//   gck_db_open      core.NewDB(dbpath, fs.NewDisk(), time, cfg)   core/db.go:90-108
//                      path.Join(cfg.DataDir, dbpath)              core/db.go:91
//                      Disk.Open: createDir, ReadDir, active file  internal/fs/disk.go:50-68,80-120
//                      db.init -> FS.Walk (lexical, recursive)     core/db.go:110-123, disk.go:122-145
//                      replay on the GPU (gck_replay)              replaces core/db.go:125-178
//   gck_db_open_mem  InMemory FS: one file "data", also active     internal/fs/memory.go:46-80
//   gck_db_get       DB.Get -> get: lazy CRC on read               core/db.go:287-316
//   gck_db_keys      DB.Keys                                       core/db.go:318-324
//
// The keydir (core/keydir.go) is filled from the replay tuples in walk order:
// set overwrites, tombstones delete, lastOffset = final_last_offset.
#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gocask_hip.h"

namespace {

// CRC-32/IEEE for the read path (Get's lazy check, core/db.go:311).  Replay never
// calls this: its verdicts come from the device pipeline.
uint32_t crc32_host(const uint8_t *p, uint64_t n) {
    struct Table {  // built once, thread-safe (a function-local static's initializer)
        uint32_t t[256];
        Table() {
            for (uint32_t i = 0; i < 256; ++i) {
                uint32_t c = i;
                for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
                t[i] = c;
            }
        }
    };
    static const Table tab;
    const uint32_t *T = tab.t;
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < n; ++i) c = T[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return ~c;
}

struct KdEntry {  // kdEntry (core/keydir.go:3-9)
    uint32_t crc, ts, value_pos, value_size;
    uint32_t file;
};

struct Mapped {
    std::string path, name;
    const uint8_t *data = nullptr;
    uint64_t len = 0;
    void unmap() {
        if (data && len) munmap(const_cast<uint8_t *>(data), len);
        data = nullptr;
    }
};

// path.Join + path.Clean (Go "path" package semantics for slash paths).
std::string path_join(const std::string &a, const std::string &b) {
    std::string s = a.empty() ? b : (b.empty() ? a : a + "/" + b);
    if (s.empty()) return "";
    const bool rooted = s[0] == '/';
    std::vector<std::string> parts;
    size_t i = 0;
    while (i <= s.size()) {
        size_t j = s.find('/', i);
        if (j == std::string::npos) j = s.size();
        std::string p = s.substr(i, j - i);
        if (p.empty() || p == ".") {
        } else if (p == "..") {
            if (!parts.empty() && parts.back() != "..") parts.pop_back();
            else if (!rooted) parts.push_back("..");
        } else {
            parts.push_back(p);
        }
        i = j + 1;
    }
    std::string out = rooted ? "/" : "";
    for (size_t k = 0; k < parts.size(); ++k) out += (k ? "/" : "") + parts[k];
    return out.empty() ? "." : out;
}

std::string base_no_ext(const std::string &path) {  // DiskFile.Name (internal/fs/disk.go:23-27)
    size_t sl = path.find_last_of('/');
    std::string b = sl == std::string::npos ? path : path.substr(sl + 1);
    size_t dot = b.find_last_of('.');
    return dot == std::string::npos ? b : b.substr(0, dot);
}

std::string ext_of(const std::string &path) {  // path.Ext
    for (size_t i = path.size(); i-- > 0;) {
        if (path[i] == '/') break;
        if (path[i] == '.') return path.substr(i);
    }
    return "";
}

std::vector<std::string> read_dir_sorted(const std::string &dir, int &err) {
    std::vector<std::string> names;
    DIR *d = opendir(dir.c_str());
    err = 0;
    if (!d) {
        err = errno;
        return names;
    }
    while (dirent *e = readdir(d)) {
        if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
        names.push_back(e->d_name);
    }
    closedir(d);
    std::sort(names.begin(), names.end());  // os.ReadDir / filepath.Walk sort by name
    return names;
}

int mkdir_all(const std::string &p) {
    std::string cur;
    for (size_t i = 0; i <= p.size(); ++i) {
        if (i == p.size() || p[i] == '/') {
            if (!cur.empty() && cur != "/") {
                if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return -1;
            }
        }
        if (i < p.size()) cur += p[i];
    }
    return 0;
}

// filepath.Walk: lexical order, recursive, Lstat (no symlinked dirs followed).
int walk(const std::string &path, std::vector<std::string> &out) {
    struct stat st;
    if (lstat(path.c_str(), &st) != 0) return GCK_EIO;
    if (!S_ISDIR(st.st_mode)) {
        if (ext_of(path) == ".csk") out.push_back(path);
        return GCK_OK;
    }
    int err;
    auto names = read_dir_sorted(path, err);
    if (err) return GCK_EIO;
    for (auto &n : names) {
        int rc = walk(path + "/" + n, out);
        if (rc) return rc;
    }
    return GCK_OK;
}

void set_err(char *buf, size_t len, const char *msg) {
    if (buf && len) snprintf(buf, len, "%s", msg);
}

}  // namespace

struct gck_db {
    std::string path;          // dbpath after path.Join(DataDir, dbpath)
    std::string active;        // active file Name()
    bool in_memory = false;
    std::vector<uint8_t> mem;  // InMemory FS bytes
    std::vector<std::string> file_names;
    std::unordered_map<std::string, KdEntry> kd;
    std::vector<const std::string *> keys;
    uint32_t last_offset = 0;
    std::vector<uint8_t> val;
};

static int fill_keydir(gck_db *db, const std::vector<Mapped> &files, const gck_opts *opts, char *errbuf,
                       size_t errlen) {
    std::vector<gck_file> gf(files.size());
    for (size_t i = 0; i < files.size(); ++i) {
        gf[i].data = files[i].data;
        gf[i].len = files[i].len;
        gf[i].reset_after = files[i].name != db->active;  // core/db.go:117
        db->file_names.push_back(files[i].name);
    }
    gck_result res;
    int rc = gck_replay(gf.data(), (uint32_t)gf.size(), opts, &res);
    if (rc != GCK_OK && rc != GCK_EUNEXPECTED_EOF) {
        set_err(errbuf, errlen, "gocask: device replay failed (no gfx950 device?)");
        return rc;
    }
    for (uint64_t i = 0; i < res.n; ++i) {  // keyDir.set / unset in walk order
        const gck_rec &r = res.recs[i];
        const uint8_t *kp = files[r.file].data + r.rec_off + 16;
        std::string key(reinterpret_cast<const char *>(kp), r.key_len);
        if (r.flags & GCK_F_TOMBSTONE) db->kd.erase(key);
        else db->kd[key] = KdEntry{r.crc, r.ts, r.value_pos, r.value_size, r.file};
    }
    db->last_offset = res.final_last_offset;
    gck_result_free(&res);
    if (rc == GCK_EUNEXPECTED_EOF) set_err(errbuf, errlen, "gocask: startup error: unexpected EOF");
    return rc;
}

extern "C" {

int gck_db_open(const char *db_path, const gck_config *cfg, const gck_opts *opts, gck_db **out, char *errbuf,
                size_t errlen) {
    if (!out || !db_path) return GCK_EINVAL;
    *out = nullptr;
    std::string path = path_join(cfg && cfg->data_dir ? cfg->data_dir : "./", db_path);
    // Disk.createDir (internal/fs/disk.go:105-120)
    struct stat st;
    if (stat(path.c_str(), &st) != 0) {
        if (errno != ENOENT || mkdir_all(path) != 0) {
            set_err(errbuf, errlen, strerror(errno));
            return GCK_EIO;
        }
    } else if (!S_ISDIR(st.st_mode)) {
        set_err(errbuf, errlen, "file exists and it's not a folder");
        return GCK_ENOT_DIR;
    }
    // Disk.Open: active file = lexically last entry, or a new data_<n>_<unix>.csk
    int err;
    auto entries = read_dir_sorted(path, err);
    if (err) {
        set_err(errbuf, errlen, strerror(err));
        return GCK_EIO;
    }
    std::string active_file = entries.empty() ? "" : entries.back();
    if (active_file.empty()) {
        char nm[96];
        snprintf(nm, sizeof nm, "data_%zu_%lld.csk", entries.size(), (long long)time(nullptr));
        active_file = nm;
    }
    int fd = open((path + "/" + active_file).c_str(), O_RDWR | O_CREAT | O_APPEND, 0755);
    if (fd < 0) {
        std::string m = std::string("could not open db: ") + strerror(errno);
        set_err(errbuf, errlen, m.c_str());
        return GCK_EIO;
    }
    close(fd);
    gck_db *db = new gck_db();
    db->path = path;
    db->active = base_no_ext(active_file);
    std::vector<std::string> paths;
    int rc = walk(path, paths);
    std::vector<Mapped> files;
    for (auto &p : paths) {
        if (rc) break;
        Mapped m;
        m.path = p;
        m.name = base_no_ext(p);
        int f = open(p.c_str(), O_RDONLY);
        if (f < 0) {
            rc = GCK_EIO;
            break;
        }
        struct stat fs;
        fstat(f, &fs);
        m.len = (uint64_t)fs.st_size;
        if (m.len) {
            void *a = mmap(nullptr, m.len, PROT_READ, MAP_PRIVATE, f, 0);
            if (a == MAP_FAILED) {
                close(f);
                rc = GCK_EIO;
                break;
            }
            m.data = static_cast<const uint8_t *>(a);
        }
        close(f);
        files.push_back(m);
    }
    if (rc) {
        for (auto &m : files) m.unmap();
        set_err(errbuf, errlen, "gocask: walk failed");
        delete db;
        return rc;
    }
    rc = fill_keydir(db, files, opts, errbuf, errlen);
    for (auto &m : files) m.unmap();
    if (rc != GCK_OK && rc != GCK_EUNEXPECTED_EOF) {
        delete db;
        return rc;
    }
    *out = db;  // like NewDB: the DB is returned together with a startup error
    return rc;
}

int gck_db_open_mem(const uint8_t *data, uint64_t len, const gck_opts *opts, gck_db **out, char *errbuf,
                    size_t errlen) {
    if (!out || (len && !data)) return GCK_EINVAL;
    *out = nullptr;
    gck_db *db = new gck_db();
    db->in_memory = true;
    db->active = "data";
    db->mem.assign(data, data + len);
    Mapped m;
    m.name = "data";
    m.data = db->mem.data();
    m.len = len;
    std::vector<Mapped> files{m};
    int rc = fill_keydir(db, files, opts, errbuf, errlen);
    if (rc != GCK_OK && rc != GCK_EUNEXPECTED_EOF) {
        delete db;
        return rc;
    }
    *out = db;
    return rc;
}

int gck_db_get(gck_db *db, const uint8_t *key, uint32_t klen, const uint8_t **val, uint64_t *vlen) {
    if (!db || !val || !vlen) return GCK_EINVAL;
    if (klen == 0 || !key) return GCK_EINVALID_KEY;  // core/db.go:295-297
    auto it = db->kd.find(std::string(reinterpret_cast<const char *>(key), klen));
    if (it == db->kd.end()) return GCK_EKEY_NOT_FOUND;
    const KdEntry &e = it->second;
    db->val.assign(e.value_size, 0);
    if (db->in_memory) {  // InMemory.ReadFileAt: copy(b, i.b[offset:])
        if (e.value_pos > db->mem.size()) return GCK_EIO;
        const uint64_t n = std::min<uint64_t>(e.value_size, db->mem.size() - e.value_pos);
        if (n) memcpy(db->val.data(), db->mem.data() + e.value_pos, n);
    } else {  // Disk.ReadFileAt: open <path>/<File>.csk, ReadAt (short read -> error)
        const std::string p = db->path + "/" + db->file_names[e.file] + ".csk";
        int fd = open(p.c_str(), O_RDONLY);
        if (fd < 0) return GCK_EIO;
        ssize_t got = e.value_size ? pread(fd, db->val.data(), e.value_size, e.value_pos) : 0;
        close(fd);
        if (got != (ssize_t)e.value_size) return GCK_EIO;
    }
    if (e.crc != crc32_host(db->val.data(), db->val.size())) return GCK_ECRC_FAILED;  // core/db.go:311
    *val = db->val.data();
    *vlen = db->val.size();
    return GCK_OK;
}

uint64_t gck_db_keys(gck_db *db) {
    if (!db) return 0;
    db->keys.clear();
    for (auto &kv : db->kd) db->keys.push_back(&kv.first);
    return db->keys.size();
}

int gck_db_key(gck_db *db, uint64_t i, const uint8_t **key, uint32_t *klen) {
    if (!db || !key || !klen || i >= db->keys.size()) return GCK_EINVAL;
    *key = reinterpret_cast<const uint8_t *>(db->keys[i]->data());
    *klen = (uint32_t)db->keys[i]->size();
    return GCK_OK;
}

int gck_db_entry(gck_db *db, const uint8_t *key, uint32_t klen, uint32_t *crc, uint32_t *ts, uint32_t *value_pos,
                 uint32_t *value_size, const char **file) {
    if (!db) return GCK_EINVAL;
    auto it = db->kd.find(std::string(reinterpret_cast<const char *>(key), klen));
    if (it == db->kd.end()) return GCK_EKEY_NOT_FOUND;
    const KdEntry &e = it->second;
    if (crc) *crc = e.crc;
    if (ts) *ts = e.ts;
    if (value_pos) *value_pos = e.value_pos;
    if (value_size) *value_size = e.value_size;
    if (file) *file = db->file_names[e.file].c_str();
    return GCK_OK;
}

uint32_t gck_db_last_offset(gck_db *db) { return db ? db->last_offset : 0; }
const char *gck_db_active_file(gck_db *db) { return db ? db->active.c_str() : ""; }
uint32_t gck_db_nfiles(gck_db *db) { return db ? (uint32_t)db->file_names.size() : 0; }
const char *gck_db_file_name(gck_db *db, uint32_t i) {
    return db && i < db->file_names.size() ? db->file_names[i].c_str() : "";
}
void gck_db_close(gck_db *db) { delete db; }

}  // extern "C"

/* TEST INFRASTRUCTURE ONLY.  gck_replay / gck_result_free for the sanitizer
 * build of the host mirror (db.cpp): the records come from the oracle's CPU
 * restatement (orc_replay), so db.cpp's walk, mmap, keydir fill and Get run
 * under ASan/UBSan without a GPU.  Never linked into libgocask_hip.so. */
#include <stdlib.h>
#include <string.h>

#include "gocask_hip.h"
#include "gocask_oracle.h"

int gck_replay(const gck_file *files, uint32_t nfiles, const gck_opts *opts, gck_result *out) {
    (void)opts;
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    orc_file *of = calloc(nfiles ? nfiles : 1, sizeof(orc_file));
    if (!of) return GCK_ENOMEM;
    for (uint32_t i = 0; i < nfiles; ++i) {
        of[i].data = files[i].data;
        of[i].len = files[i].len;
        of[i].reset_after = files[i].reset_after;
    }
    orc_status st;
    orc_replay(of, nfiles, 1, NULL, 0, &st);
    orc_rec *recs = malloc((st.n_recs ? st.n_recs : 1) * sizeof(orc_rec));
    if (!recs) {
        free(of);
        return GCK_ENOMEM;
    }
    orc_replay(of, nfiles, 1, recs, st.n_recs, &st);
    free(of);
    out->recs = (gck_rec *)recs; /* byte-identical layouts (40 B) */
    out->n = st.n_recs;
    for (uint64_t i = 0; i < st.n_recs; ++i) out->n_crc_fail += !(recs[i].flags & ORC_F_CRC_OK);
    out->final_last_offset = st.final_last_offset;
    out->status = st.status == ORC_EUNEXPECTED_EOF ? GCK_EUNEXPECTED_EOF : GCK_OK;
    out->err_file = st.err_file;
    out->files_walked = st.files_walked;
    out->err_off = st.err_off;
    return out->status;
}

void gck_result_free(gck_result *res) {
    if (!res) return;
    free(res->recs);
    res->recs = NULL;
    res->n = 0;
}

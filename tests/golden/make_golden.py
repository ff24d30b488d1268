"""Generate the golden replay fixtures under tests/golden/<case>/.

Each fixture restates the INPUT of one of the reference's own replay tests
(files built with the reference's canonical encoder, core/testutil/utils.go:10-19,
in the walk order its mock FS yields, core/testutil/fs.go:143-178) and records
the EXPECTED answer that test asserts.  Where a test only asserts part of the
keydir, extra fields derived by hand from the reference code are stored under
"derived" with the reference lines they follow.

The encoder here is an independent few-line restatement of testutil.Entry
(zlib.crc32 == Go hash/crc32 IEEE); expected values are NOT produced by the
oracle, so the oracle can be checked against them.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import struct
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))


def entry(now, key, val):
    return struct.pack("<IIII", zlib.crc32(val), now, len(key), len(val)) + key + val


def tomb(now, key):
    return struct.pack("<IIII", zlib.crc32(key), now, 0, len(key)) + key


def write_case(name, files, walk, active, expect, note, derived=None, status="ok", final_last_offset=None):
    d = os.path.join(HERE, name)
    os.makedirs(d, exist_ok=True)
    for fn in os.listdir(d):
        os.remove(os.path.join(d, fn))
    for fname, data in files.items():
        with open(os.path.join(d, fname + ".csk"), "wb") as f:
            f.write(data)
    meta = dict(walk=walk, active=active, expect=expect, note=note, status=status)
    if derived:
        meta["derived"] = derived
    if final_last_offset is not None:
        meta["final_last_offset"] = final_last_offset
    with open(os.path.join(d, "case.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


def main():
    # core/db_test.go:140-279 TestShould_Fetch_Existing_Values_After_Startup
    seed = [("data0", "foo", "foo bar baz", 1234), ("data0", "name", "john doe", 443),
            ("data01", "foo1", "foo bar baz", 1234), ("data01", "name1", "john doe", 443),
            ("data02", "1234", '{"foo": "bar"}', 34389), ("data03", "foo bar baz", "test", 999999),
            ("data03", "foo bar baz 01", "test", 999999), ("data03", "foo2", "test foo bar", 200),
            ("data03", "foo bar baz 02", "test", 999999), ("data03", "baz", "test", 999999)]
    files, walk = {}, []
    for f, k, v, t in seed:
        if f not in files:
            files[f] = b""
            walk.append(f)
        files[f] += entry(t, k.encode(), v.encode())
    expect = {k: {"value": v, "file": f} for f, k, v, t in seed}
    write_case("existing_after_startup", files, walk, "data", expect,
               "core/db_test.go:140-279: every Get after NewDB returns its value")

    # core/db_test.go:281-352 TestShould_Fetch_Updated_Values_From_Different_Files
    seed = [("data", "foo", "foo bar baz", 1234), ("data0", "bar", "foo bar baz", 1234),
            ("data01", "foo", "john doe overwrites you", 443), ("data02", "bar", "foo bar buzzed", 1234)]
    files, walk = {}, []
    for f, k, v, t in seed:
        if f not in files:
            files[f] = b""
            walk.append(f)
        files[f] += entry(t, k.encode(), v.encode())
    write_case("updated_values_across_files", files, walk, "data",
               {"foo": {"value": "john doe overwrites you", "file": "data01"},
                "bar": {"value": "foo bar buzzed", "file": "data02"}},
               "core/db_test.go:281-352: last writer (walk order) wins across files",
               derived={"foo": {"value_pos": 19}, "bar": {"value_pos": 19},
                        "_why": "core/keydir.go:25; data02 follows data01 which is not active -> reset"})

    # core/db_test.go:375-393 TestShould_Not_Be_Able_To_Retrieve_Deleted_Key_After_Startup
    # in-memory FS: single file "data" that is also the active file (internal/fs/memory.go:46-74)
    d = entry(12345, b"foo", b"bar") + tomb(12345, b"foo")
    write_case("deleted_after_startup", {"data": d}, ["data"], "data", {},
               "core/db_test.go:375-393: Get(foo) after re-open -> ErrKeyNotFound",
               final_last_offset=41)

    # core/db_test.go:428-471 TestShould_Fetch_All_Keys_In_Order
    seed = [("data", "foo"), ("data", "bar"), ("data01", "foobar"), ("data02", "baz")]
    files, walk = {}, []
    for f, k in seed:
        if f not in files:
            files[f] = b""
            walk.append(f)
        files[f] += entry(123, k.encode(), b"val")
    write_case("keys_in_order", files, walk, "data",
               {k: {"file": f} for f, k in seed},
               "core/db_test.go:428-471: Keys() == {foo, bar, foobar, baz}",
               derived={"foo": {"value_pos": 19, "crc": 2548021861, "ts": 123, "value_size": 3},
                        "bar": {"value_pos": 41}, "foobar": {"value_pos": 66}, "baz": {"value_pos": 19},
                        "_why": "data is the active file and walked first, so its lastOffset (44) "
                                "carries into data01 (core/db.go:117-119, core/keydir.go:25)"},
               final_last_offset=0)

    # core/db_test.go:473-492 TestShould_Not_Fetch_Removed_Keys (in-memory)
    d = (entry(12345, b"foo", b"val") + entry(12345, b"baz", b"val") + entry(12345, b"bar", b"val")
         + tomb(12345, b"baz"))
    write_case("removed_keys", {"data": d}, ["data"], "data",
               {"foo": {"value": "val"}, "bar": {"value": "val"}},
               "core/db_test.go:473-492: Keys() == {foo, bar}")

    # core/db_test.go:494-500 TestShould_Return_Empty_Keys_Slice_For_Empty_DB
    write_case("empty_db", {"data": b""}, ["data"], "data", {},
               "core/db_test.go:494-500: Keys() == []", final_last_offset=0)

    # core/db_test.go:738-757 TestShould_Fail_CRC_Check: the stored CRC is of
    # "uncorrupted" but the 11 value bytes read back are "corrupted" + 2 zero
    # bytes (WithMockValue copies 9 bytes into an 11-byte buffer, fs.go:37-49)
    hdr = struct.pack("<IIII", zlib.crc32(b"uncorrupted"), 12345, 3, 11)
    write_case("crc_fail", {"data": hdr + b"foo" + b"corrupted\x00\x00"}, ["data"], "data",
               {"foo": {"crc_ok": False}},
               "core/db_test.go:738-757: Get -> ErrCRCFailed (the verdict is a reject)")

    # Partial write (core/testutil/memory.go:18-29, core/db_test.go:616-649): the
    # second entry lost its last byte; the reference never replays it.  Go
    # stdlib semantics give: "key" is inserted (Discard borrows a byte of the
    # next header), the next header is read one byte late, its key length is
    # 0x06000000 and io.ReadFull hits EOF -> io.ErrUnexpectedEOF -> startup error.
    d = (entry(12345, b"user", b"user123456") + entry(12345, b"key", b"foobarbaz")[:-1]
         + entry(12345, b"ishould", b"befine"))
    write_case("partial_write_desync", {"data": d}, ["data"], "data",
               {"user": {"value": "user123456"}},
               "derived: core/db.go:145-170 + io.ReadFull semantics -> gocask: startup error: unexpected EOF",
               derived={"err_off": 58, "n_recs": 2}, status="unexpected_eof")

    # db_test.go:39-74 writeReadAndAssert over testdata/data.txt: 1000 Puts into
    # one file; every key's Get returns the last value written for it.
    lines = [l for l in open(os.path.join(HERE, "data.txt")).read().split("\n") if l]
    d = b""
    exp = {}
    for l in lines:
        k, v = l.split("|")[0], l.split("|")[1]
        d += entry(12345, k.encode(), v.encode())
        exp[k] = {"value": v}
    write_case("datatxt_1000_puts", {"data": d}, ["data"], "data", exp,
               "db_test.go:39-74: 1000 Puts of testdata/data.txt, 858 live keys")

    # EOF classes (Go stdlib semantics), derived:
    base = entry(7, b"k1", b"v1")
    write_case("eof_partial_header", {"data": base + b"\x01" * 7}, ["data"], "data",
               {"k1": {"value": "v1"}}, "derived: 1-15 trailing header bytes -> ErrUnexpectedEOF",
               status="unexpected_eof", derived={"err_off": len(base)})
    write_case("eof_header_only", {"data": base + struct.pack("<IIII", 0, 7, 5, 5)}, ["data"], "data",
               {"k1": {"value": "v1"}}, "derived: header then EOF -> io.EOF on the key read (clean stop)")
    write_case("eof_partial_key", {"data": base + struct.pack("<IIII", 0, 7, 5, 5) + b"ab"}, ["data"],
               "data", {"k1": {"value": "v1"}}, "derived: partial key -> ErrUnexpectedEOF",
               status="unexpected_eof", derived={"err_off": len(base)})
    write_case("eof_short_value", {"data": base + entry(7, b"k2", b"value2")[:-2]}, ["data"], "data",
               {"k1": {"value": "v1"}}, "derived: short value -> Discard io.EOF, record dropped, clean stop")
    write_case("empty_key_tombstone", {"data": base + struct.pack("<IIII", 0, 7, 0, 0) + entry(8, b"k3", b"")},
               ["data"], "data", {"k1": {"value": "v1"}, "k3": {"value": ""}},
               "derived: header{KeySize 0, ValueSize 0} is a tombstone of the empty key; replay continues")


if __name__ == "__main__":
    main()

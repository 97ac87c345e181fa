#!/usr/bin/env python3
"""Per-kernel static ISA statistics from a `hipcc --cuda-device-only -S` listing: instruction
counts by class, lane-write/read (SGPR spill traffic), scratch accesses, and the register/spill
fields of the .amdhsa descriptor and the .set lines.

    usage: tools/isa_stats.py listing.s [substring ...]
"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\w+):\s*;\s*@", text, re.M):
        name = m.group(1)
        end = text.find(".Lfunc_end", m.end())
        body = text[m.end():end]
        ins = [l.strip() for l in body.split("\n") if l.startswith("\t") and not l.strip().startswith((".", ";"))]
        meta = {}
        for k in ("num_vgpr", "num_sgpr", "private_seg_size"):
            mm = re.search(r"\.set %s\.%s, (\d+)" % (re.escape(name), k), text)
            if mm:
                meta[k] = int(mm.group(1))
        yield name, ins, meta


def stats(ins):
    c = {
        "total": len(ins),
        "valu": sum(1 for l in ins if l.startswith("v_") and not l.startswith(("v_readlane", "v_writelane"))),
        "salu": sum(1 for l in ins if l.startswith("s_") and not l.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch", "s_load", "s_buffer"))),
        "writelane": sum(1 for l in ins if l.startswith("v_writelane")),
        "readlane": sum(1 for l in ins if l.startswith("v_readlane")),
        "scratch": sum(1 for l in ins if l.startswith(("scratch_", "buffer_"))),
        "ds": sum(1 for l in ins if l.startswith("ds_")),
        "global": sum(1 for l in ins if l.startswith("global_")),
        "f64": sum(1 for l in ins if "_f64" in l.split()[0]),
    }
    return c


def main():
    text = open(sys.argv[1]).read()
    subs = sys.argv[2:]
    for name, ins, meta in kernels(text):
        if subs and not any(s in name for s in subs):
            continue
        print(name[:90], meta, stats(ins))


if __name__ == "__main__":
    main()

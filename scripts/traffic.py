#!/usr/bin/env python3
"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/traffic.json entries.

HBM bytes per launch of KernelEntry = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM) -- the output read-modify-write here is exactly that access
(16 B per lane), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
usage: traffic.py KEY SUMMARY_JSON [profiles/traffic.json]
"""
import json
import os
import sys

key, summ = sys.argv[1], sys.argv[2]
out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                        "profiles", "traffic.json")
s = json.load(open(summ))
ks = [k for k in s if "kernel_entry" in k and "true, false" in k or ("kernel_entry" in k and k.endswith("false>(rtk::KernelArgs)"))]
k = [k for k in s if "kernel_entry" in k and "FETCH_SIZE" in s[k] and "WRITE_SIZE" in s[k] and k.rstrip(")").endswith("false>(rtk::KernelArgs")]
if not k:
    k = [k for k in s if "kernel_entry" in k and "FETCH_SIZE" in s[k]]
k = k[0]
fetch, write = s[k]["FETCH_SIZE"], s[k]["WRITE_SIZE"]
hbm = (2.0 * fetch + write) * 1024.0
db = json.load(open(out)) if os.path.exists(out) else {}
db[key] = {"hbm_bytes_per_launch": int(hbm), "fetch_size_kib": fetch, "write_size_kib": write, "kernel": k,
           "note": "(2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 FETCH_SIZE correction"}
for c, name in (("SQ_INSTS_VALU", "valu_insts_per_launch"), ("SQ_INSTS_LDS", "lds_insts_per_launch"),
                ("SQ_INSTS_SALU", "salu_insts_per_launch"), ("GRBM_GUI_ACTIVE", "gui_active_cycles_all_xcds")):
    if c in s[k]:
        db[key][name] = int(s[k][c])
json.dump(db, open(out, "w"), indent=1, sort_keys=True)
print(key, db[key])

"""Critical-path statistics of traced exact GS-CF flow passes (diagnostic builds, lab only).

    make BUILD=build_trace LIBDIR=amg_amd/lib_trace EXTRA=-DSSS_GS_TRACE
    SSS_AMG_LIB=amg_amd/lib_trace/libsss_amg.so SSS_GS_TRACE_FILE=/tmp/t.bin python tools/gs_level_times.py ...
    python tools/gs_trace_stats.py /tmp/t.bin

Per traced pass (rows, depth): the median time between the last publish of depth d-1 and of depth
d (the critical step), the median staging time of a row (ticket -> products staged), how often a
row had its products staged before its previous depth finished, and the median time from the
previous depth's last publish to the row's own publish.  Stamps: s_memrealtime (100 MHz).
"""
import sys

import numpy as np


def passes(path):
    b = open(path, "rb").read()
    o = 0
    while o < len(b):
        nrows, depth = np.frombuffer(b, np.int32, 2, o)
        o += 8
        h_off = np.frombuffer(b, np.int32, depth + 1, o)
        o += 4 * (depth + 1)
        tr = np.frombuffer(b, np.uint64, 4 * nrows, o).reshape(nrows, 4).astype(np.int64)
        o += 8 * 4 * nrows
        yield int(nrows), int(depth), h_off, tr


for nrows, depth, h_off, tr in passes(sys.argv[1]):
    if nrows == 0 or tr[:, 2].max() == 0:
        continue
    d_of = np.repeat(np.arange(depth), np.diff(h_off))
    pub = np.full(depth, 0, np.int64)
    np.maximum.at(pub, d_of, tr[:, 2])
    step = np.diff(pub)
    stage = tr[:, 1] - tr[:, 0]
    prev = np.concatenate([[tr[:, 0].min()], pub[:-1]])[d_of]
    early = np.mean(tr[:, 1] <= prev)
    after = tr[:, 2] - prev
    span = (pub[-1] - tr[:, 0].min()) / 100.0
    print(f"rows {nrows:7d} depth {depth:5d} len {np.median(tr[:, 3]):7.0f}  pass {span:9.1f} us  step median "
          f"{np.median(step) / 100:6.2f} us  staging median {np.median(stage) / 100:6.2f} us  staged before deps "
          f"{100 * early:5.1f} %  publish after deps median {np.median(after) / 100:6.2f} us")

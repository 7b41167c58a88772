"""Known-byte streams for calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 (tools/profile.sh).

MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read;
other widths are uncalibrated.  This runs, on 1 GiB buffers (well past the 256 MiB Infinity Cache),
one read-only stream at 4, 8 and 16 B per lane (gs_stream_read) and one write-only stream at 4, 8 and
16 B per lane (gs_stream_write), each launched once; tools/pmc_summary.py divides the known bytes by the
counters of these launches to get the factor for each access width.
"""

from __future__ import annotations

import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

CAL_BYTES = 1 << 30


def main():
    import torch

    from aiocluster_amd import _lib

    L = _lib.load()
    dev = torch.device("cuda", 0)
    src = torch.empty(CAL_BYTES, dtype=torch.uint8, device=dev).fill_(7)
    dst = torch.empty(CAL_BYTES, dtype=torch.uint8, device=dev)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    P = C.c_void_p
    for w in (4, 8, 16):
        assert L.gs_stream_read(P(src.data_ptr()), CAL_BYTES, w, P(sink.data_ptr()), P(stream.cuda_stream)) == 0
        torch.cuda.synchronize(dev)
    for w in (4, 8, 16):
        assert L.gs_stream_write(P(dst.data_ptr()), CAL_BYTES, w, P(stream.cuda_stream)) == 0
        torch.cuda.synchronize(dev)
    print(json.dumps({"cal_bytes": CAL_BYTES, "launches": ["read4", "read8", "read16", "write4", "write8", "write16"]}))


if __name__ == "__main__":
    main()

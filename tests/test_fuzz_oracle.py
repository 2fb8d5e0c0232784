"""The two CPU restatements agree on mutated frames (tests/fuzzframes.py): per-frame classes, every
field of every session record (pyoracle.record_to_row), the DNS side records and the batch stats,
under each filter -- the oracle the GPU fuzz test (test_gpu_fuzz.py) checks against is itself
cross-checked on inputs far from the synthetic distribution."""
import numpy as np
import pytest

import fuzzframes
from oracle import coracle, pyoracle


@pytest.mark.parametrize("flt", [0, 1, 2])
def test_fuzz_c_vs_python_oracle(flt):
    frames, offs = fuzzframes.generate(3000, seed=11 + flt)
    out, dns, cls, st = coracle.parse_classify(coracle.make_cfg(flt), frames, offs)
    pcfg = pyoracle.Config.from_bitmap(coracle.default_bitmap(), session_filter=flt)
    classes, records, pdns, pst = pyoracle.run_batch(pcfg, frames, offs)
    assert classes == cls.tolist()
    assert len(records) == len(out)
    for r, row in zip(records, out):
        want = pyoracle.record_to_row(r)
        for k, v in want.items():
            got = row[k].tolist() if isinstance(v, list) else int(row[k])
            assert got == v, (k, got, v, int(row["pkt_index"]))
    assert [(int(d["pkt_index"]), int(d["payload_offset"]), int(d["payload_length"])) for d in dns] == \
        [(a, b, c) for a, b, c, _, _ in pdns]
    for k, v in pst.items():
        assert int(st[0][k]) == v, k
    # the mutations reach every class the filter allows
    assert set(classes) == ({0, 1, 2} if flt == 2 else {0, 1, 2, 3})

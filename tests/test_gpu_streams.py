"""Several tracked sequences on one GPU at once (tools/serve_streams.py): independent
contexts, each with its own stream and graphs, enqueued round-robin.  Every stream's
per-frame {bestp, cost} must be bit-identical to the same stream tracked alone — no
state is shared between contexts (testmodel.cpp:117-139 per stream)."""
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))


def test_concurrent_streams_equal_alone():
    import serve_streams
    sts = serve_streams.make_streams(3, 7, P=64, G=6)
    try:
        hist = serve_streams.check_against_alone(sts, list(range(6)))
        assert all(h.shape == (6, 27) for h in hist)
        # the streams track different sequences: their results differ
        assert not (hist[0] == hist[1]).all()
    finally:
        for st in sts:
            st["ctx"].close()

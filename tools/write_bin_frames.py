"""Write a synthetic sequence as MSRA-style frames (000000_depth.bin ...: headerless
float32 mm, 240 x 320), the layout observedmodel::load_data reads -- for exercising the
recorded-frame paths (bench.py --frames, hpe_track --frames).
usage: write_bin_frames.py OUT_DIR N [seed]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "tests"), str(ROOT / "hand-pose-estimation_amd")]
import numpy as np  # noqa: E402

import hand_data  # noqa: E402
import oracle_np  # noqa: E402

out, n = Path(sys.argv[1]), int(sys.argv[2])
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
out.mkdir(parents=True, exist_ok=True)
geo, rad = hand_data.geometry_cm()
hand = oracle_np.Hand(geo, rad)
for f, th in enumerate(hand_data.trajectory(n, seed=seed)):
    oracle_np.render_depth_mm(hand, th).astype("<f4").tofile(out / f"{f:06d}_depth.bin")
print(f"{n} frames in {out}")

"""Golden pad amounts of the REFERENCE InputPadder (core/utils/utils.py:7-24).

Run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_padder_golden.py
Records ``_pad`` and the padded / unpadded shapes for the BASELINE image sizes
and a few ragged ones, in both modes, into tests/golden/padder.json.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
DIMS = [(436, 1024), (375, 1242), (368, 496), (1080, 1920), (17, 23), (8, 8), (1, 1)]


def main() -> None:
    sys.path.insert(0, "/root/reference/core")
    import torch
    from utils.utils import InputPadder   # the reference's own class
    out = []
    for h, w in DIMS:
        for mode in ("sintel", "kitti"):
            p = InputPadder((1, 3, h, w), mode=mode)
            x = torch.arange(3 * h * w, dtype=torch.float32).reshape(1, 3, h, w)
            (y,) = p.pad(x)
            out.append({"dims": [h, w], "mode": mode, "pad": list(p._pad),
                        "padded": list(y.shape[-2:]), "corner_sum": float(y[..., :2, :2].sum()),
                        "roundtrip": bool(torch.equal(p.unpad(y), x))})
    (HERE / "padder.json").write_text(json.dumps(out, indent=1))
    print(len(out), "cases")


if __name__ == "__main__":
    main()

"""Pack the reference's Mouse semi-supervised split into one .npz for GPU boxes.

Data only (no reference code): the cached split datasources/temp_data/
Mouse_100_500_0.3.json (semiTrain 100 = 30 labeled + 70 unlabeled, valid 500)
and its 600 PNGs under data/pose/mouse/croppeds_bbox/images, read with PIL and
flipped to BGR (the reference reads them with cv2.imread, utils/process.py:86-88).
The pack is written to data/mouse_100_500_0.3.npz (git-ignored; it travels to
the GPU box with the tree, ~70 MB).  Run in the build container, where the
reference tree exists:

    python tools/pack_mouse.py [/root/reference]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ubpl-poseestimation_amd"))

from ubpl_amd.mouse import MouseData, PACK_NAME  # noqa: E402


def main(ref="/root/reference"):
    src = MouseData(root=os.path.join(ref, "data", "pose", "mouse", "croppeds_bbox"),
                    split_dir=os.path.join(ref, "datasources", "temp_data"))
    out = os.path.join(ROOT, "data", PACK_NAME)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    src.write_pack(out, 100, 500, 0.3)
    print("wrote", out, os.path.getsize(out) // (1 << 20), "MiB")


if __name__ == "__main__":
    main(*sys.argv[1:])

"""Digest of the device layout every test world converts to (host only).

rtow_scene_check with RTOW_LAYOUT_DUMP=path writes every array
rtow_scene_upload would copy to the GPU (rtow_device.hip / rtow_layout.cpp:
buildLayout) plus the layout's scalars; this hashes that dump for the
product's scene builders and every golden fixture, with the SAH and the
reference tree.  Two builds whose digests agree upload the same bytes, so a
host-side refactor of the conversion can be checked on the CPU.

  python tools/layout_digest.py > digests.txt
"""
import glob
import hashlib
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-one-weekend_amd"))
import rtow  # noqa: E402

BUILDS = [("three_sphere", 1, "none"), ("random_ned", 100, "synthetic"), ("random_ned", 487, "synthetic"),
          ("cornell", 1, "none"), ("cornell_smoke", 1, "none"), ("final_ned", 1, "synthetic"),
          ("random", 100, "none"), ("cornell_box", 1, "none")]


def worlds():
    for name, n, img in BUILDS:
        yield f"{name}/{n}", rtow.Scene.build(name, n=n, image=img, scene_seed=1)
    for path in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "*.scn"))):
        yield os.path.basename(path), rtow.Scene.load(path)


def main():
    dump = os.path.join(tempfile.mkdtemp(), "layout.bin")
    os.environ["RTOW_LAYOUT_DUMP"] = dump
    for label, sc in worlds():
        for tree in ("sah", "ref"):
            if tree == "ref":
                os.environ["RTOW_BVH"] = "ref"
            else:
                os.environ.pop("RTOW_BVH", None)
            try:
                sc.check()
                h = hashlib.sha256(open(dump, "rb").read()).hexdigest()[:16]
            except rtow.RtowError as e:
                h = f"error {e.code}"
            print(f"{label:28s} {tree} {h}")
    os.environ.pop("RTOW_BVH", None)


if __name__ == "__main__":
    main()

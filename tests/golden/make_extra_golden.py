#!/usr/bin/env python3
"""Golden fixtures beyond the BASELINE configs, from the REFERENCE ITSELF
(oracle/_ref, the reference's headers unmodified):

* dof_*: the depth-of-field camera path (RTOW_FLAG_CAMERA_DOF), rendered by
  oracle/_ref/ref_harness_dof -- the same harness as make_golden.py's,
  compiled with CAMERA_DOF_EN 1 (camera.h:124-126);
* medium_bvh: ConstantMedium below a BvhNode (ref_harness.cpp mediumBvhNed:
  the reference's classes, media in the BVH, one in an n == 1 node);
* medium_nested: a medium whose boundary is a medium, and one whose boundary
  is a list holding a medium (ref_harness.cpp mediumNestedNed);
* medium_bvh_wrapped: media below a BvhNode behind a Translate, inside a list
  and behind RotateY(Translate(...)) (ref_harness.cpp mediumBvhWrappedNed);
* tie_bvh_entry: a list item and a BvhNode item tied at a t where the
  BvhNode's box is entered exactly (ref_harness.cpp tieBvhEntryNed);
* random_ref, random_ref_noimg, cornell_box: the reference's own non-NED
  builders randomScene() (scenes.h:29-120; with its earth1300x1300.jpg, the
  harness run in the reference's directory, and without it: the glass
  fallback) and cornellBox() (scenes.h:220-353), called directly.

Writes <case>.{scn,lin,bgra} (texels stripped, as make_golden.py), the
cameras, and manifest_extra.json (`flags`: the rtow_params flags the case
renders with).

Usage: python3 tests/golden/make_extra_golden.py   (after make -C oracle ref)
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
HARNESS_DOF = os.path.join(REPO, "oracle", "_ref", "ref_harness_dof")

sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
from make_golden import strip_texels, write_png  # noqa: E402
from scene_io import synthetic_image  # noqa: E402

FLAG_CAMERA_DOF = 2  # include/rtow.h
# name, harness, flags, harness scene, n, image mode, W, H, spp, render seed
CASES = [
    ("dof_three_sphere", HARNESS_DOF, FLAG_CAMERA_DOF, "three_sphere", 100, "none", 64, 36, 16, 3),
    ("dof_random100", HARNESS_DOF, FLAG_CAMERA_DOF, "random_ned", 100, "synthetic", 48, 27, 16, 5),
    ("medium_bvh", HARNESS, 0, "medium_bvh", 100, "none", 64, 36, 64, 9),
    ("medium_nested", HARNESS, 0, "medium_nested", 100, "none", 64, 36, 64, 11),
    ("medium_bvh_wrapped", HARNESS, 0, "medium_bvh_wrapped", 100, "none", 64, 36, 64, 13),
    ("tie_bvh_entry", HARNESS, 0, "tie_bvh_entry", 100, "none", 64, 36, 16, 15),
    ("random_ref", HARNESS, 0, "random", 100, "reference", 64, 36, 16, 17),
    ("random_ref_noimg", HARNESS, 0, "random", 100, "none", 48, 27, 16, 19),
    ("cornell_box", HARNESS, 0, "cornell_box", 100, "none", 48, 48, 64, 21),
]
REF_DIR = "/root/reference/rayTracingOneWeekend"  # its input_images/ (read only)
SCENE_SEED = 1


def main():
    if not (os.path.exists(HARNESS) and os.path.exists(HARNESS_DOF)):
        sys.exit("build the harnesses first: make -C oracle ref")
    tmp = tempfile.mkdtemp(prefix="rtow_dof_")
    dirs = {"none": os.path.join(tmp, "none"), "synthetic": os.path.join(tmp, "synth"), "reference": REF_DIR}
    os.makedirs(dirs["none"])
    os.makedirs(os.path.join(dirs["synthetic"], "input_images"))
    write_png(os.path.join(dirs["synthetic"], "input_images", "1_earth_8k.jpg"), synthetic_image(2048, 1024))
    env = dict(os.environ, RTOW_SCENE_SEED=str(SCENE_SEED))
    manifest = {"scene_seed": SCENE_SEED, "generator": "oracle/_ref/ref_harness[_dof]", "cases": []}
    for name, harness, flags, scene, n, img, W, H, spp, seed in CASES:
        raw = os.path.join(tmp, name + ".scn")
        subprocess.run([harness, "dump", scene, raw, "--n", str(n), "--cwd", dirs[img]], env=env, check=True,
                       capture_output=True)
        sha, ntex, hdr = strip_texels(raw, os.path.join(HERE, name + ".scn"))
        subprocess.run([harness, "render", scene, str(W), str(H), str(spp), os.path.join(HERE, name),
                        "--n", str(n), "--seed", str(seed), "--cwd", dirs[img]], env=env, check=True)
        subprocess.run([HARNESS, "camera", str(W), str(H), os.path.join(HERE, f"cam_{W}x{H}.cam")], env=env,
                       check=True)
        manifest["cases"].append(dict(name=name, harness=os.path.basename(harness), flags=flags, scene=scene, n=n, image=img, width=W, height=H, spp=spp, seed=seed,
                                      texel_bytes=ntex, texel_sha256=sha, n_hitables=hdr[2]))
        print(f"{name}: {hdr[2]} hitables")
    # keep the cases other generators add (make_graze_golden.py: graze_medium)
    mpath = os.path.join(HERE, "manifest_extra.json")
    ours = {c[0] for c in CASES}
    if os.path.exists(mpath):
        manifest["cases"] += [c for c in json.load(open(mpath))["cases"] if c["name"] not in ours]
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()

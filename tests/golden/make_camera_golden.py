#!/usr/bin/env python3
"""Golden cameras after the GUI frame loop's updates, from the REFERENCE's own
Camera (setOrientationMatrix camera.h:231-235 + setLookFromPoint, basis by
setCamera_QuaternionMatrix camera.h:315-342), via oracle/_ref/ref_harness
camera_oriented.  Writes tests/golden/cam_oriented_<k>.cam and
cameras_oriented.json (the inputs); and the look-at cameras of
setCamera_Euler (camera.h:271-313, ref_harness camera_euler) as
cam_euler_<k>.cam and cameras_euler.json.
Usage: python3 tests/golden/make_camera_golden.py"""
import json
import math
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
HARNESS = os.path.join(HERE, "..", "..", "oracle", "_ref", "ref_harness")


def rows_yaw_pitch(yaw_deg, pitch_deg):
    """view (w), east (u), down (v) rows of the NED start basis w=(-1,0,0),
    u=(0,1,0), v=(0,0,-1) turned by yaw about down, then pitch about east."""
    cy, sy = math.cos(math.radians(yaw_deg)), math.sin(math.radians(yaw_deg))
    cp, sp = math.cos(math.radians(pitch_deg)), math.sin(math.radians(pitch_deg))
    w = (-cy * cp, -sy * cp, sp)
    u = (-sy, cy, 0.0)
    v = (-cy * sp, -sy * sp, -cp)
    return [round(x, 7) for x in w + u + v]


CASES = [
    (64, 36, [0.0, 0.0, 0.0], rows_yaw_pitch(0, 0)),
    (64, 36, [-20.0, 5.0, -3.0], rows_yaw_pitch(25, 0)),
    (48, 48, [100.0, -50.0, -20.0], rows_yaw_pitch(-40, 12)),
]


# look_from, look_at, up, vfov, aspect, aperture, focus distance, t0, t1
EULER = [
    ([13.0, 2.0, 3.0], [0.0, 0.0, 0.0], [0.0, 1.0, 0.0], 20.0, 16.0 / 9.0, 0.1, 10.0, 0.0, 1.0),  # book 1's cover
    ([0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, -1.0], 60.0, 1920.0 / 1080.0, 2.0, 1000.0, 0.0, 1.0),  # main.cpp's
    ([478.0, 278.0, -600.0], [278.0, 278.0, 0.0], [0.0, 1.0, 0.0], 40.0, 1.0, 0.0, 10.0, 0.0, 1.0),  # book 2's
    ([0.0, 5.0, 0.0], [0.0, 0.0, 0.0], [0.0, 1.0, 0.0], 45.0, 1.5, 0.5, 5.0, 0.25, 0.75),  # up along the view: u = 0
]


def main():
    eul = []
    for k, (lf, la, up, fov, asp, ap, fd, t0, t1) in enumerate(EULER):
        path = os.path.join(HERE, f"cam_euler_{k}.cam")
        vals = lf + la + up + [fov, asp, ap, fd, t0, t1]
        subprocess.run([HARNESS, "camera_euler"] + [repr(float(x)) for x in vals] + [path], check=True)
        eul.append({"look_from": lf, "look_at": la, "up": up, "vfov": fov, "aspect": asp, "aperture": ap,
                    "focus": fd, "t0": t0, "t1": t1, "file": os.path.basename(path)})
    with open(os.path.join(HERE, "cameras_euler.json"), "w") as f:
        json.dump(eul, f, indent=1)
    out = []
    for k, (W, H, lf, rows) in enumerate(CASES):
        path = os.path.join(HERE, f"cam_oriented_{k}.cam")
        args = [HARNESS, "camera_oriented", str(W), str(H)] + [repr(float(x)) for x in lf + rows] + [path]
        subprocess.run(args, check=True)
        out.append({"width": W, "height": H, "look_from": lf, "rows": rows, "file": os.path.basename(path)})
    with open(os.path.join(HERE, "cameras_oriented.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

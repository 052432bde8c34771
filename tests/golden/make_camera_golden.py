"""Generate tests/golden/camera_controls.json with the reference's own
camera.hpp (oracle/_ref/camera_driver, built by oracle/ref/Makefile from
/root/reference/include).  Runs only where /root/reference exists.

    python tests/golden/make_camera_golden.py
"""
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
DRIVER = os.path.join(REPO, "oracle", "_ref", "camera_driver")

ASPECT = "0x1.c71c72p+0"      # float(1920) / float(1080)
# (kind, a, b): 0 init (Cornell camera, main.cpp:199-202), 1 rotate, 2 translate, 3 fov
OPS = [(0, 0, 0), (1, 12, -7), (1, -3.5, 2), (2, 4, 9), (3, -1, 0), (3, 50, 0), (1, 0, 140), (1, 0, -149.75),
       (2, -0.5, -0.25), (3, 3, 0), (1, 300, 0), (1, 37.25, 61.5), (3, -44.5, 0), (3, -0.25, 0), (2, 123, -77),
       (0, 0, 0), (1, 1, 1), (1, -1, -1)]
INIT = ["0 2.8 7 0 2.8 0 0 1 0 45 " + ASPECT, "0 5 5 0 0 0 0 1 0 60 1"]


def main():
    if not os.path.exists(DRIVER):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle", "ref")], check=True)
    lines, inits = [], iter(INIT)
    for k, a, b in OPS:
        lines.append(f"{k} {a} {b}")
        if k == 0:
            lines.append(next(inits))
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "ops.txt"), os.path.join(d, "out.txt")
        open(src, "w").write("\n".join(lines) + "\n")
        subprocess.run([DRIVER, src, dst], check=True, stdout=subprocess.DEVNULL)
        rows = [[float.fromhex(t) for t in ln.split()] for ln in open(dst) if ln.strip()]
    json.dump({"ops": OPS, "init": INIT, "states": [[r.hex() for r in row] for row in rows]},
              open(os.path.join(HERE, "camera_controls.json"), "w"))
    print(len(rows), "states")


if __name__ == "__main__":
    main()

"""Copy the texture PNGs that data/assets/materials.yaml names from a reference
checkout's data/ directory into data/textures/ (untracked: asset data, ~55 MB).

    python tools/fetch_textures.py [/root/reference/data]

The library and vxpt_offline load them when present (vxpt_load_textures); the
tests use synthetic textures and do not need these files.
"""
import os
import re
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data"
    names = set(re.findall(r"textures/[\w.\-]+\.png", open(os.path.join(REPO, "data", "assets", "materials.yaml")).read()))
    os.makedirs(os.path.join(REPO, "data", "textures"), exist_ok=True)
    n = 0
    for rel in sorted(names):
        s, d = os.path.join(src, rel), os.path.join(REPO, "data", rel)
        if os.path.exists(s):
            shutil.copyfile(s, d)
            n += 1
        else:
            print("missing", s)
    print("copied %d of %d textures" % (n, len(names)))


if __name__ == "__main__":
    main()

"""Pack / unpack the accuracy-parity data cache (data_cache/avmnist_real_pairs, made by
scripts/accuracy_parity.py prepare from the reference's own sample files) for the GPU box: the float32
spectrograms are byte-shuffled and zlib-compressed (1.7x; the box receives the whole tree on every call).

  python scripts/acc_pack.py pack     # here: data_cache/ -> data_pack/
  python scripts/acc_pack.py unpack   # on the box: data_pack/ -> data_cache/
"""
import os
import shutil
import sys
import zlib

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "data_cache", "avmnist_real_pairs")
DST = os.path.join(REPO, "data_pack", "avmnist_real_pairs")


def pack():
    for split in ("train", "test"):
        os.makedirs(os.path.join(DST, split), exist_ok=True)
        for f in os.listdir(os.path.join(SRC, split)):
            src = os.path.join(SRC, split, f)
            if f.endswith(".f32"):
                a = np.fromfile(src, dtype=np.uint8)
                with open(os.path.join(DST, split, f + ".zs"), "wb") as fh:
                    fh.write(zlib.compress(a.reshape(-1, 4).T.copy().tobytes(), 1))
            else:
                shutil.copy(src, os.path.join(DST, split, f))


def unpack():
    for split in ("train", "test"):
        os.makedirs(os.path.join(SRC, split), exist_ok=True)
        for f in os.listdir(os.path.join(DST, split)):
            src = os.path.join(DST, split, f)
            if f.endswith(".zs"):
                raw = np.frombuffer(zlib.decompress(open(src, "rb").read()), dtype=np.uint8)
                raw.reshape(4, -1).T.copy().tofile(os.path.join(SRC, split, f[:-3]))
            else:
                shutil.copy(src, os.path.join(SRC, split, f))


if __name__ == "__main__":
    {"pack": pack, "unpack": unpack}[sys.argv[1]]()

"""PNG fixtures for tests/test_png.py: the reference's own 4x3 test.png (data,
copied as is) and its decode under the reference's rules (PIL 8-bit RGBA,
alpha forced to 0 for RGB files as png_set_filler(0) does,
src/png_decoder.cpp:94-97; then byte / 255.0f, src/image.cpp:70).
Runs only where /root/reference is mounted:  python tests/golden/make_png_golden.py"""
import os
import shutil

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
src = "/root/reference/test.png"
shutil.copyfile(src, os.path.join(HERE, "test.png"))
raw = Image.open(src)
e = np.asarray(raw.convert("RGBA")).astype(np.int64)
if raw.mode == "RGB":
    e[..., 3] = 0
np.save(os.path.join(HERE, "png_test.npy"), e.astype(np.float32) / np.float32(255.0))
print("wrote test.png, png_test.npy", raw.mode, raw.size)

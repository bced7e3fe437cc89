"""Import helper: the package directory name holds '-' characters, so it is put on sys.path."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "sccg-genome-compression_amd")
if PKG_DIR not in sys.path:
    sys.path.insert(0, PKG_DIR)

import sccg  # noqa: E402,F401

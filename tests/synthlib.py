"""Re-export of the package's synthetic-pair generator binding for the tests."""
from pkg import PKG_DIR  # noqa: F401  (puts the package directory on sys.path)
from synth import PROFILES, synth_pair  # noqa: F401

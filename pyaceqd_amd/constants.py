"""Physical constants and module-level configuration (mirrors pyaceqd/constants.py:1-3)."""
hbar = 0.6582119569  # meV*ps
pybind_path = ""     # unused: no ACEutils; kept so `constants.pybind_path` lookups keep working
temp_dir = ""        # unused: libpqd takes in-memory arguments, no temp files are written

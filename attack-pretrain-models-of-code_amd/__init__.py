"""apmc_amd — MI355X-native victim-query engine for ALERT (attack-pretrain-models-of-code).

Drop-in for the reference's query hot path: `Model.get_results` (victim scoring of mutant
batches), the mutant construction + featurisation that feeds it, the greedy / GA / MHM-NS attack
drivers that issue it, and the masked-LM substitute generation.  Device work runs in the gfx950
HIP kernels of `csrc/` behind the C-ABI `include/alert_engine.h` (lib/libalert_engine.so).
"""
import pathlib

PKG_DIR = pathlib.Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "lib" / "libalert_engine.so"
# the same sources built with -DAE_TOOLS: timing / A-B entry points (ae_bench_*) and AE_* knobs
TOOLS_LIB_PATH = PKG_DIR / "lib" / "libalert_engine_tools.so"
HOSTLIB_PATH = PKG_DIR / "lib" / "libalert_host.so"
DATA_DIR = PKG_DIR.parent / "data"

__version__ = "0.1.0"

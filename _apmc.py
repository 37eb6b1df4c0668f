"""Registers the product package directory `attack-pretrain-models-of-code_amd/` (a name that is
not a Python identifier) as the importable package `apmc_amd`.  Import this module first:

    import _apmc            # noqa: F401
    from apmc_amd.model import Model
"""
import importlib.util
import pathlib
import sys

PKG_DIR = pathlib.Path(__file__).resolve().parent / "attack-pretrain-models-of-code_amd"


def load():
    mod = sys.modules.get("apmc_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "apmc_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["apmc_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


load()

"""Load the product package (directory name is not a Python identifier)."""
import importlib.util
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cpu-based-ray-tracer_amd")


def load():
    spec = importlib.util.spec_from_file_location("rt_amd", os.path.join(PKG, "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


rt = load()

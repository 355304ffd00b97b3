"""Import alias for the package directory `laplace-dqn-snake-game_amd/`.

The directory name carries hyphens, so it cannot be imported by name; this
shim loads it as the package `snake_amd` (`import snake_amd`).
"""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "laplace-dqn-snake-game_amd")
_spec = importlib.util.spec_from_file_location("snake_amd", os.path.join(_DIR, "__init__.py"),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["snake_amd"] = _mod
_spec.loader.exec_module(_mod)

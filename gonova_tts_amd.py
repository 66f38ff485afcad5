"""Import shim: exposes the hyphenated package directory `gonova-tts_amd/` as the
importable package `gonova_tts_amd` (a hyphen is not a legal Python identifier).

Python treats a module that defines ``__path__`` as a package, so
``import gonova_tts_amd.engine`` resolves submodules inside ``gonova-tts_amd/``.
"""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "gonova-tts_amd")]
__package__ = __name__
_init = _os.path.join(__path__[0], "__init__.py")
with open(_init, "r", encoding="utf-8") as _f:
    exec(compile(_f.read(), _init, "exec"), globals())

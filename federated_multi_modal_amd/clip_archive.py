"""Read the tensors of a CLIP checkpoint without executing anything from the file.

load_clip_to_cpu (trainers/maple.py:21-40) opens the checkpoint clip._download fetched with
torch.jit.load and takes model.state_dict().  Those official files are TorchScript archives (a zip
holding data.pkl, code/ and data/<storage>); torch.load(weights_only=True) refuses them, and
torch.jit.load would compile and run the archive's code.  This module reads such an archive the way a
weights-only loader reads a plain checkpoint: data.pkl is unpickled with an allow-list of exactly the
constructs a TorchScript module tree uses --

  * `__torch__.*` classes: an inert record that keeps the attribute dict handed to BUILD (no class
    code, no __setstate__ of the archive's own);
  * torch._utils._rebuild_tensor_v2 and torch.<Type>Storage: tensors rebuilt here from the raw
    little-endian storage records data/<key> of the zip;
  * collections.OrderedDict (the empty backward-hook dicts);

-- anything else raises pickle.UnpicklingError.  The module tree is then walked into a flat
{dotted.name: tensor} dict, the keys model.state_dict() has (parameters and registered buffers).

Plain state dicts saved with torch.save go through torch.load(weights_only=True) unchanged; its errors
propagate (corrupt files are not retried with another loader)."""
from __future__ import annotations

import collections
import io
import pickle
import zipfile
from typing import Dict

import torch

_STORAGE_DTYPES = {"DoubleStorage": torch.float64, "FloatStorage": torch.float32, "HalfStorage": torch.float16,
                   "BFloat16Storage": torch.bfloat16, "LongStorage": torch.int64, "IntStorage": torch.int32,
                   "ShortStorage": torch.int16, "CharStorage": torch.int8, "ByteStorage": torch.uint8,
                   "BoolStorage": torch.bool}


class _ScriptRecord:
    """Stand-in for one TorchScript object: BUILD stores its attribute dict, nothing else runs."""

    def __setstate__(self, state):
        self.__dict__["state"] = state


class _StorageType:
    def __init__(self, dtype):
        self.dtype = dtype


def _rebuild_tensor(storage, offset, size, stride, requires_grad=False, hooks=None, *extra):
    t = storage.as_strided(tuple(size), tuple(stride), int(offset)).clone()
    return t


class _ArchiveUnpickler(pickle.Unpickler):
    def __init__(self, data: bytes, zf: zipfile.ZipFile, prefix: str):
        super().__init__(io.BytesIO(data))
        self.zf, self.prefix = zf, prefix
        self._storages: Dict[str, torch.Tensor] = {}

    def find_class(self, module, name):
        if module.startswith("__torch__"):
            return _ScriptRecord
        if module == "torch._utils" and name == "_rebuild_tensor_v2":
            return _rebuild_tensor
        if module == "torch" and name in _STORAGE_DTYPES:
            return _StorageType(_STORAGE_DTYPES[name])
        if module == "collections" and name == "OrderedDict":
            return collections.OrderedDict
        raise pickle.UnpicklingError(f"{module}.{name} is not allowed in a CLIP TorchScript archive")

    def persistent_load(self, pid):
        if not (isinstance(pid, tuple) and len(pid) >= 5 and pid[0] == "storage"):
            raise pickle.UnpicklingError(f"unexpected persistent id {pid!r}")
        stype, key = pid[1], str(pid[2])
        if not isinstance(stype, _StorageType):
            raise pickle.UnpicklingError(f"unexpected storage type {stype!r}")
        if key not in self._storages:
            raw = bytearray(self.zf.read(f"{self.prefix}/data/{key}"))
            self._storages[key] = torch.frombuffer(raw, dtype=stype.dtype) if raw else torch.empty(0, dtype=stype.dtype)
        return self._storages[key]


def is_torchscript_archive(path: str) -> bool:
    """A zip whose top directory holds code/ (TorchScript) rather than only data.pkl + data/ (torch.save)."""
    if not zipfile.is_zipfile(path):
        return False
    with zipfile.ZipFile(path) as zf:
        return any("/code/" in n for n in zf.namelist())


def read_torchscript_state_dict(path: str) -> Dict[str, torch.Tensor]:
    """{name: tensor} of every tensor attribute in the archive's module tree (model.state_dict()'s keys)."""
    with zipfile.ZipFile(path) as zf:
        names = zf.namelist()
        pkl = [n for n in names if n.count("/") == 1 and n.endswith("/data.pkl")]
        if len(pkl) != 1:
            raise ValueError(f"{path}: not a TorchScript archive (no top-level data.pkl)")
        prefix = pkl[0].split("/")[0]
        order = f"{prefix}/byteorder"
        if order in names and zf.read(order).decode().strip() != "little":
            raise ValueError(f"{path}: big-endian archive")
        root = _ArchiveUnpickler(zf.read(pkl[0]), zf, prefix).load()
    out: Dict[str, torch.Tensor] = {}

    def walk(obj, pre):
        state = obj.__dict__.get("state", {}) if isinstance(obj, _ScriptRecord) else {}
        if not isinstance(state, dict):
            return
        for k, v in state.items():
            if isinstance(v, torch.Tensor):
                out[pre + k] = v
            elif isinstance(v, _ScriptRecord):
                walk(v, pre + k + ".")
    walk(root, "")
    return out


def load_clip_state_dict(path: str) -> Dict[str, torch.Tensor]:
    """The CLIP weights in `path`: a TorchScript archive (read as above) or a torch.save'd state dict /
    {"state_dict": ...} checkpoint (torch.load with weights_only=True)."""
    if is_torchscript_archive(path):
        return read_torchscript_state_dict(path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd:
        sd = sd["state_dict"]
    return sd

"""Config surface of the reference (lib/config/default.py:17-127) without yacs.

`CfgNode` implements the subset of yacs.config.CfgNode the training path uses:
attribute and item access, merge_from_file (YAML, safe loader), merge_from_list
(CLI `KEY VALUE` pairs with literal parsing), freeze / defrost, per-node
`new_allowed`, and yacs' type checking on merge.
"""
import ast
import copy

import yaml

_VALID = (tuple, list, str, int, float, bool, type(None))


class CfgNode(dict):
    IMMUTABLE = "__immutable__"
    NEW_ALLOWED = "__new_allowed__"

    def __init__(self, init=None, new_allowed=False):
        super().__init__()
        self.__dict__[CfgNode.IMMUTABLE] = False
        self.__dict__[CfgNode.NEW_ALLOWED] = new_allowed
        for k, v in (init or {}).items():
            self[k] = CfgNode(v, new_allowed) if isinstance(v, dict) and not isinstance(
                v, CfgNode) else v

    def __getattr__(self, name):
        if name in self:
            return self[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if self.is_frozen():
            raise AttributeError(f"Attempted to set {name} to {value}, but CfgNode is immutable")
        self[name] = value

    def __deepcopy__(self, memo):
        out = CfgNode(new_allowed=self.is_new_allowed())
        for k, v in self.items():
            out[k] = copy.deepcopy(v, memo)
        return out

    def clone(self):
        return copy.deepcopy(self)

    def is_frozen(self):
        return self.__dict__[CfgNode.IMMUTABLE]

    def is_new_allowed(self):
        return self.__dict__[CfgNode.NEW_ALLOWED]

    def _set_immutable(self, flag):
        self.__dict__[CfgNode.IMMUTABLE] = flag
        for v in self.values():
            if isinstance(v, CfgNode):
                v._set_immutable(flag)

    def freeze(self):
        self._set_immutable(True)

    def defrost(self):
        self._set_immutable(False)

    # ---- merging ----
    def merge_from_file(self, path):
        with open(path, "r") as f:
            data = yaml.safe_load(f) or {}
        self.merge_from_other_cfg(CfgNode(data))

    def merge_from_other_cfg(self, other):
        _merge(other, self, [])

    def merge_from_list(self, opts):
        if not opts:
            return
        if len(opts) % 2:
            raise ValueError(f"Override list has odd length: {opts}")
        for key, val in zip(opts[0::2], opts[1::2]):
            node = self
            parts = key.split(".")
            for p in parts[:-1]:
                if p not in node:
                    raise KeyError(f"Non-existent config key: {key}")
                node = node[p]
            last = parts[-1]
            if last not in node and not node.is_new_allowed():
                raise KeyError(f"Non-existent config key: {key}")
            v = _decode(val)
            if last in node:
                v = _coerce(v, node[last], key)
            node[last] = v

    def __str__(self):
        def fmt(node, indent):
            lines = []
            for k in sorted(node):
                v = node[k]
                if isinstance(v, CfgNode):
                    lines.append(" " * indent + f"{k}:")
                    lines.extend(fmt(v, indent + 2))
                else:
                    lines.append(" " * indent + f"{k}: {v}")
            return lines
        return "\n".join(fmt(self, 0))

    def dump(self):
        def plain(n):
            return {k: plain(v) if isinstance(v, CfgNode) else v for k, v in n.items()}
        return yaml.safe_dump(plain(self))


def _decode(v):
    if isinstance(v, dict):
        return CfgNode(v)
    if not isinstance(v, str):
        return v
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        return v


def _coerce(new, old, key):
    if type(new) is type(old) or old is None or new is None:
        return new
    if isinstance(old, tuple) and isinstance(new, list):
        return tuple(new)
    if isinstance(old, list) and isinstance(new, tuple):
        return list(new)
    if isinstance(old, float) and isinstance(new, int) and not isinstance(new, bool):
        return float(new)
    if isinstance(old, str) and isinstance(new, (int, float)):
        return str(new)
    raise ValueError(f"Type mismatch ({type(old)} vs. {type(new)}) with values ({old} vs. {new}) "
                     f"for config key: {key}")


def _merge(src, dst, path):
    for k, v in src.items():
        full = ".".join(path + [k])
        v = _decode(v) if not isinstance(v, CfgNode) else v
        if k in dst:
            if isinstance(dst[k], CfgNode):
                if not isinstance(v, CfgNode):
                    raise ValueError(f"Type mismatch for config key {full}: expected a node")
                v.__dict__[CfgNode.NEW_ALLOWED] = dst[k].is_new_allowed()
                _merge(v, dst[k], path + [k])
            else:
                dst[k] = _coerce(v, dst[k], full)
        elif dst.is_new_allowed():
            dst[k] = v
        else:
            raise KeyError(f"Non-existent config key: {full}")

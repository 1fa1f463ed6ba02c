"""Flag registry: one declaration serves both the CLI and the library API.

Mirrors the role of ``tcb/flags.py:36-89`` (ParamSpec registry that doubles as
absl flags), but absl is not part of this stack, so the command-line parser is
our own: it accepts ``--name=value``, ``--name value``, bare ``--name`` /
``--noname`` for booleans, comma lists for list flags, and rejects positional
arguments (the reference rejects them to catch ``--distortions False`` typos,
``tcb/tf_cnn_benchmarks.py:39-46``).
"""

from __future__ import annotations

import collections
from typing import Any, Dict, Iterable, List, Optional, Sequence

ParamSpec = collections.namedtuple(
    "ParamSpec", ["flag_type", "default_value", "description", "kwargs"])

# name -> ParamSpec, in declaration order.
param_specs: "collections.OrderedDict[str, ParamSpec]" = collections.OrderedDict()


def _register(name: str, spec: ParamSpec) -> None:
    param_specs[name] = spec


def DEFINE_string(name, default, help):  # noqa: N802  (keeps the familiar spelling)
    _register(name, ParamSpec("string", default, help, {}))


def DEFINE_boolean(name, default, help):  # noqa: N802
    _register(name, ParamSpec("boolean", default, help, {}))


def DEFINE_integer(name, default, help, lower_bound=None, upper_bound=None):  # noqa: N802
    _register(name, ParamSpec("integer", default, help,
                              {"lower_bound": lower_bound, "upper_bound": upper_bound}))


def DEFINE_float(name, default, help, lower_bound=None, upper_bound=None):  # noqa: N802
    _register(name, ParamSpec("float", default, help,
                              {"lower_bound": lower_bound, "upper_bound": upper_bound}))


def DEFINE_enum(name, default, enum_values, help):  # noqa: N802
    _register(name, ParamSpec("enum", default, help, {"enum_values": list(enum_values)}))


def DEFINE_list(name, default, help):  # noqa: N802
    _register(name, ParamSpec("list", default, help, {}))


class FlagError(ValueError):
    """Raised for malformed command lines."""


_TRUE = {"1", "true", "t", "yes", "y", "on"}
_FALSE = {"0", "false", "f", "no", "n", "off"}


def _convert(name: str, spec: ParamSpec, raw: str) -> Any:
    t = spec.flag_type
    try:
        if t == "string":
            return raw
        if t == "boolean":
            low = raw.lower()
            if low in _TRUE:
                return True
            if low in _FALSE:
                return False
            raise FlagError("flag --%s expects a boolean, got %r" % (name, raw))
        if t == "integer":
            return int(raw, 0) if raw.lower().startswith(("0x", "0o", "0b")) else int(raw)
        if t == "float":
            return float(raw)
        if t == "enum":
            if raw not in spec.kwargs["enum_values"]:
                raise FlagError("flag --%s value %r not in %s"
                                % (name, raw, spec.kwargs["enum_values"]))
            return raw
        if t == "list":
            return [s for s in raw.split(",") if s] if raw else []
    except ValueError as e:
        if isinstance(e, FlagError):
            raise
        raise FlagError("flag --%s: cannot parse %r as %s" % (name, raw, t)) from e
    raise FlagError("unknown flag type %s" % t)


def _check_bounds(name: str, spec: ParamSpec, value: Any) -> None:
    if value is None or spec.flag_type not in ("integer", "float"):
        return
    lo, hi = spec.kwargs.get("lower_bound"), spec.kwargs.get("upper_bound")
    if lo is not None and value < lo:
        raise FlagError("flag --%s=%s is below its lower bound %s" % (name, value, lo))
    if hi is not None and value > hi:
        raise FlagError("flag --%s=%s is above its upper bound %s" % (name, value, hi))


def parse_flags(argv: Sequence[str],
                specs: Optional[Dict[str, ParamSpec]] = None,
                allow_unknown: bool = False) -> Dict[str, Any]:
    """Parses ``argv`` (without the program name) into ``{name: value}``.

    Only flags that appear on the command line are returned; callers merge
    them over the defaults.  ``--help``/``-h`` raises SystemExit after printing
    the flag table.
    """
    specs = specs if specs is not None else param_specs
    out: Dict[str, Any] = {}
    i = 0
    argv = list(argv)
    while i < len(argv):
        tok = argv[i]
        i += 1
        if tok in ("-h", "--help", "--helpfull"):
            print(format_help(specs))
            raise SystemExit(0)
        if tok == "--":
            rest = argv[i:]
            if rest:
                raise FlagError("Received unknown positional arguments: %s" % rest)
            break
        if not tok.startswith("-"):
            raise FlagError("Received unknown positional arguments: %s" % [tok])
        body = tok.lstrip("-")
        if "=" in body:
            name, raw = body.split("=", 1)
            has_value = True
        else:
            name, raw, has_value = body, None, False
        spec = specs.get(name)
        if spec is None and name.startswith("no") and name[2:] in specs \
                and specs[name[2:]].flag_type == "boolean" and not has_value:
            out[name[2:]] = False
            continue
        if spec is None:
            if allow_unknown:
                if not has_value and i < len(argv) and not argv[i].startswith("-"):
                    i += 1
                continue
            raise FlagError("Unknown command line flag '%s'" % name)
        if spec.flag_type == "boolean" and not has_value:
            out[name] = True
            continue
        if not has_value:
            if i >= len(argv):
                raise FlagError("flag --%s requires a value" % name)
            raw = argv[i]
            i += 1
        value = _convert(name, spec, raw)
        _check_bounds(name, spec, value)
        out[name] = value
    return out


def format_help(specs: Optional[Dict[str, ParamSpec]] = None) -> str:
    specs = specs if specs is not None else param_specs
    lines = ["flags:"]
    for name, spec in specs.items():
        extra = ""
        if spec.flag_type == "enum":
            extra = " <%s>" % "|".join(str(v) for v in spec.kwargs["enum_values"])
        lines.append("  --%s%s: %s\n    (default: %r)" % (name, extra, spec.description,
                                                          spec.default_value))
    return "\n".join(lines)


def to_argv(values: Dict[str, Any], specs: Optional[Dict[str, ParamSpec]] = None) -> List[str]:
    """Inverse of :func:`parse_flags` for non-default values (used by the
    distributed test runner to re-launch a Params tuple as a process,
    cf. ``tcb/benchmark_cnn_distributed_test.py:43-58``)."""
    specs = specs if specs is not None else param_specs
    argv = []
    for name, value in values.items():
        spec = specs[name]
        if value == spec.default_value:
            continue
        if value is None:
            continue
        if spec.flag_type == "boolean":
            argv.append("--%s" % name if value else "--no%s" % name)
        elif spec.flag_type == "list":
            argv.append("--%s=%s" % (name, ",".join(str(v) for v in value)))
        else:
            argv.append("--%s=%s" % (name, value))
    return argv


def names() -> Iterable[str]:
    return param_specs.keys()

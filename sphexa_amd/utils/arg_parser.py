"""Command-line parsing with the reference's semantics.

Parity: reference main/src/io/arg_parser.hpp:30-142 — ``get(option, default)`` (numbers parsed as int if integral
else float; a value starting with '-' is not a value), ``getCommaList``, ``exists``, and the output cadence helpers
``isOutputStep``, ``isOutputTime``, ``isExtraOutputStep``, ``strBeforeSign``/``strAfterSign``/``numberAfterSign``,
``removeModifiers``.
"""

from __future__ import annotations

import re
from typing import List, Sequence

_INT = re.compile(r"^[+-]?\d+$")


def str_is_integral(s: str) -> bool:
    return bool(_INT.match(s.strip())) if s else False


class ArgParser:
    def __init__(self, argv: Sequence[str]):
        self.args = list(argv)

    def get(self, option: str, default=None):
        if option in self.args:
            i = self.args.index(option)
            if i + 1 < len(self.args) and not self.args[i + 1].startswith("-") or (
                    i + 1 < len(self.args) and _is_number(self.args[i + 1])):
                v = self.args[i + 1]
                if isinstance(default, (int, float)) and not isinstance(default, bool):
                    return int(v) if str_is_integral(v) else float(v)
                return v
        return default

    def get_comma_list(self, option: str) -> List[str]:
        v = self.get(option, "")
        return [t for t in str(v).replace(",", " ").split() if t]

    def exists(self, option: str) -> bool:
        return option in self.args


def _is_number(s: str) -> bool:
    try:
        float(s)
        return s.startswith("-") and len(s) > 1 and (s[1].isdigit() or s[1] == ".")
    except ValueError:
        return False


def is_output_step(step: int, freq: str) -> bool:
    if not str_is_integral(freq):
        return False
    f = int(freq)
    return f != 0 and step % f == 0


def is_output_time(t1: float, t2: float, freq: str) -> bool:
    f = float(freq)
    if str_is_integral(freq) or f == 0.0:
        return False
    closest = int(t2 / f) * f
    return t1 <= closest < t2


def is_extra_output_step(step: int, t1: float, t2: float, extras: Sequence[str]) -> bool:
    for tok in extras:
        if str_is_integral(tok):
            if int(tok) == step:
                return True
        else:
            t = float(tok)
            if t1 <= t < t2:
                return True
    return False


def str_before_sign(s: str, sign: str) -> str:
    p = s.find(sign)
    return s if p < 0 else s[:p]


def str_after_sign(s: str, sign: str) -> str:
    p = s.find(sign)
    return "" if p < 0 else s[p + len(sign):]


def number_after_sign(s: str, sign: str) -> int:
    a = str_after_sign(s, sign)
    return int(a) if str_is_integral(a) else -1


def remove_modifiers(init: str) -> str:
    return str_before_sign(str_before_sign(init, ":"), ",")


def stop_simulation(iteration: int, time: float, max_step: str) -> bool:
    if str_is_integral(max_step):
        return iteration >= int(max_step)
    return time > float(max_step)

"""``prime_factor`` — factorisation by trial division + Miller-Rabin + Pollard rho.

Mapped but missing in the reference (``/root/reference/ops/__init__.py:22``);
contract is new (prime_factor.CONTRACT.md; parity unpinned). Deterministic
Miller-Rabin bases make primality exact below 3.3e24.
"""
from __future__ import annotations

import math
import random
from typing import Any, Dict, List

from . import register_op
from ._common import fail, is_int, js_int

MAX_BITS = 96
_SMALL = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41]


def is_prime(n: int) -> bool:
    if n < 2:
        return False
    for p in _SMALL:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in _SMALL:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def _rho(n: int, rng: random.Random) -> int:
    if n % 2 == 0:
        return 2
    while True:
        y, c, m = rng.randrange(1, n), rng.randrange(1, n), 128
        g = q = r = 1
        x = ys = y
        while g == 1:
            x = y
            for _ in range(r):
                y = (y * y + c) % n
            k = 0
            while k < r and g == 1:
                ys = y
                for _ in range(min(m, r - k)):
                    y = (y * y + c) % n
                    q = q * abs(x - y) % n
                g = math.gcd(q, n)
                k += m
            r *= 2
        if g == n:
            g = 1
            while g == 1:
                ys = (ys * ys + c) % n
                g = math.gcd(abs(x - ys), n)
        if g != n:
            return g


def factorize(n: int) -> List[int]:
    out: List[int] = []
    for p in (2, 3, 5, 7, 11, 13):
        while n % p == 0:
            out.append(p)
            n //= p
    stack, rng = [n] if n > 1 else [], random.Random(n)
    while stack:
        m = stack.pop()
        if m == 1:
            continue
        if is_prime(m):
            out.append(m)
            continue
        d = _rho(m, rng)
        stack += [d, m // d]
    return sorted(out)


@register_op("prime_factor")
def prime_factor(payload: Any) -> Dict[str, Any]:
    payload = payload or {}
    if not isinstance(payload, dict):
        return fail("payload must be a dict")
    n = payload.get("n")
    if isinstance(n, str) and n.strip().isdigit():
        n = int(n.strip())
    if not is_int(n) or n < 1:
        return fail("payload.n must be a positive integer")
    if n.bit_length() > MAX_BITS:
        return fail(f"payload.n must be < 2**{MAX_BITS}")
    fs = factorize(n)
    return {"ok": True, "n": js_int(n), "factors": [js_int(f) for f in fs], "is_prime": n > 1 and fs == [n]}

"""Shared HTTP plumbing for the outbound ERP trigger ops (opt-in only)."""
from __future__ import annotations

import os
from datetime import datetime, timezone
from typing import Any, Dict, Optional, Tuple

TIMEOUT_SEC = float(os.getenv("ERP_HTTP_TIMEOUT_SEC", "15"))


def auth(user_var: str, pass_var: str) -> Optional[Tuple[str, str]]:
    user, pwd = os.environ.get(user_var), os.environ.get(pass_var)
    return (user, pwd) if user is not None and pwd is not None else None


def utc_now() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def post(url: str, body: Dict[str, Any], basic: Optional[Tuple[str, str]], headers: Optional[Dict[str, str]] = None):
    import requests

    return requests.post(url, json=body, auth=basic, headers=headers or {}, timeout=TIMEOUT_SEC)

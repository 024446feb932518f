"""``trigger_oracle`` — Oracle SCM Cloud "Material Issue" inventory transaction.

Behaviour of ``/root/reference/ops/trigger_oracle.py:9-35`` (POST to
``{ORACLE_HOST}/fscmRestApi/resources/11.13.18.05/inventoryTransactions`` with
basic auth ``ORA_USER``/``ORA_PASS``; ``{"status": "success", "oracle_tx_id"}``
on 201, ``{"error": ...}`` otherwise), with two fixes: the op is registered (the
reference's was dead code) but only enabled when ``TASKS`` names it explicitly
(it has external side effects), and ``TransactionDate`` is the current UTC time
(or ``payload.date``) instead of a hard-coded 2026-01-04.
"""
from __future__ import annotations

import os
from typing import Any, Dict

from . import register_op
from ._erp import auth, post, utc_now

ORACLE_HOST = os.environ.get("ORACLE_HOST", "https://eg-dev.fa.us2.oraclecloud.com")
PATH = "/fscmRestApi/resources/11.13.18.05/inventoryTransactions"


@register_op("trigger_oracle")
def trigger_oracle(payload: Dict[str, Any]) -> Dict[str, Any]:
    payload = payload or {}
    try:
        body = {
            "TransactionType": payload.get("transaction_type", "Material Issue"),
            "ItemNumber": payload.get("item"),
            "TransactionQuantity": payload.get("qty"),
            "TransactionDate": payload.get("date") or utc_now(),
        }
        r = post(ORACLE_HOST + PATH, body, auth("ORA_USER", "ORA_PASS"),
                 {"Content-Type": "application/vnd.oracle.adf.resourceitem+json"})
        if r.status_code == 201:
            return {"status": "success", "oracle_tx_id": r.json()["TransactionId"]}
        return {"error": f"Oracle Rejected: {r.text}"}
    except Exception as exc:
        return {"error": str(exc)}

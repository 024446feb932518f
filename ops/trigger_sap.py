"""``trigger_sap`` — SAP S/4HANA QualityNotification via OData.

Behaviour of ``/root/reference/ops/trigger_sap.py:9-33`` (POST to
``{SAP_HOST}/sap/opu/odata/sap/API_QUALNOTIFICATION_SRV/A_QualityNotification``
with basic auth ``SAP_USER``/``SAP_PASS``; ``{"status": "success", "sap_id"}`` on
201, ``{"error": ...}`` otherwise). Registered but opt-in (external side
effects): enabled only when ``TASKS`` names it.
"""
from __future__ import annotations

import os
from typing import Any, Dict

from . import register_op
from ._erp import auth, post

SAP_HOST = os.environ.get("SAP_HOST", "https://my-sap-instance.com")
PATH = "/sap/opu/odata/sap/API_QUALNOTIFICATION_SRV/A_QualityNotification"


@register_op("trigger_sap")
def trigger_sap(payload: Dict[str, Any]) -> Dict[str, Any]:
    payload = payload or {}
    try:
        body = {
            "NotificationType": payload.get("notification_type", "Q1"),
            "Material": payload.get("material"),
            "NotificationText": payload.get("text"),
            "Priority": str(payload.get("priority", "1")),
        }
        r = post(SAP_HOST + PATH, body, auth("SAP_USER", "SAP_PASS"))
        if r.status_code == 201:
            return {"status": "success", "sap_id": r.json()["d"]["Notification"]}
        return {"error": f"SAP Rejected: {r.text}"}
    except Exception as exc:
        return {"error": str(exc)}

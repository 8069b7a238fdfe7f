"""Registration / heartbeat client to the orchestrator (T8; reference
``src/server/server_connection.py:10-34``).

Wire behaviour kept from the reference:
  * ``POST http://{SERVER_HOST}:{SERVER_PORT}/model/register``
  * header ``api_key: <API_KEY>``
  * JSON ``{"name": NAME, "socket": "http://{ADVERTISE_HOST}:{PORT}"}``
  * 2xx -> ``connected = True``; connection error / timeout / HTTP error -> ``connected = False``
    and a debug log line, then retry.
  * keeps re-registering every ``HEARTBEAT_S`` (reference ``WAIT_TIME = 10``) until shutdown --
    it is a periodic heartbeat, not a one-shot.

Defects of the reference that are fixed (SURVEY.md C9, §2.A race notes):
  * requests carry a timeout, so a hung orchestrator cannot block shutdown forever;
  * the wait is an ``Event.wait`` -> shutdown is noticed immediately, not after a 1 s slice;
  * any other ``RequestException`` (e.g. an invalid URL when ``SERVER_PORT`` is unset) is
    logged and retried instead of silently killing the thread;
  * ``legacy_payload=True`` emits the older ``{"modelName", "modelPort"}`` body
    (``old-rev server_connection.pyc@L14-29``) for orchestrators of that vintage.
"""
from __future__ import annotations

import logging
from typing import Callable, Optional

import requests

from .api.state import ServiceState

logger = logging.getLogger("mlsamd.discovery")


def registration_url(server_host: str, server_port) -> str:
    return f"http://{server_host}:{server_port}/model/register"


def registration_payload(name: str, advertise_host: str, model_port, legacy: bool = False) -> dict:
    if legacy:
        return {"modelName": name, "modelPort": model_port}
    return {"name": name, "socket": f"http://{advertise_host}:{model_port}"}


def register_once(
    session: requests.Session,
    url: str,
    api_key: str,
    payload: dict,
    timeout: float,
    legacy: bool = False,
) -> None:
    headers = {} if legacy else {"api_key": api_key}
    r = session.post(url, headers=headers, json=payload, timeout=timeout)
    r.raise_for_status()


def register_model_to_server(
    state: ServiceState,
    server_port,
    model_port,
    model_name: str,
    api_key: str = "",
    server_host: str = "host.docker.internal",
    advertise_host: str = "host.docker.internal",
    wait_time: float = 10.0,
    timeout: float = 5.0,
    legacy_payload: bool = False,
    on_attempt: Optional[Callable[[bool], None]] = None,
) -> None:
    """Heartbeat loop; returns when ``state.shutdown`` is set."""
    url = registration_url(server_host, server_port)
    payload = registration_payload(model_name, advertise_host, model_port, legacy_payload)
    with requests.Session() as session:
        while not state.shutdown.is_set():
            ok = False
            try:
                register_once(session, url, api_key, payload, timeout, legacy_payload)
                ok = True
                state.connected = True
                state.registrations += 1
                state.last_register_error = None
            except (requests.exceptions.ConnectionError, requests.exceptions.Timeout, requests.exceptions.HTTPError) as e:
                state.connected = False
                state.last_register_error = f"{type(e).__name__}: {e}"
                logger.debug("Registering to server fails. Retry in %s seconds", wait_time)
            except requests.exceptions.RequestException as e:  # e.g. InvalidURL: keep the thread alive
                state.connected = False
                state.last_register_error = f"{type(e).__name__}: {e}"
                logger.warning("Registration request invalid (%s); retry in %s seconds", e, wait_time)
            if on_attempt is not None:
                on_attempt(ok)
            state.shutdown.wait(wait_time)
    logger.debug("[Healthcheck] Server Registration Thread Halted.")


def start_heartbeat(state: ServiceState, settings) -> "threading.Thread | None":
    """Submit the heartbeat to the background pool (reference ``main.py:82``)."""
    if not settings.REGISTER or settings.SERVER_PORT in (None, ""):
        logger.info("registration disabled (REGISTER=%s SERVER_PORT=%s)", settings.REGISTER, settings.SERVER_PORT)
        return None
    state.pool.submit(
        register_model_to_server,
        state,
        settings.SERVER_PORT,
        settings.PORT,
        settings.NAME,
        settings.API_KEY,
        settings.SERVER_HOST,
        settings.ADVERTISE_HOST,
        settings.HEARTBEAT_S,
        settings.REGISTER_TIMEOUT_S,
        bool(getattr(settings, "REGISTER_LEGACY", False)),
    )
    return None

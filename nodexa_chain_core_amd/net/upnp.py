"""UPnP port mapping (`-upnp`): ThreadMapPort of the reference (src/net.cpp:1465-1563) without
miniupnpc.

The Internet Gateway Device protocol is three small exchanges, done here with the standard
library:

  discover   SSDP M-SEARCH to 239.255.255.250:1900 (UDP multicast), answers carry a LOCATION URL
  describe   HTTP GET of that device description (XML): the WANIPConnection / WANPPPConnection
             service's controlURL; the LAN address is the local end of a connection to the device
  control    SOAP POSTs to the controlURL: GetExternalIPAddress (the node advertises it,
             AddLocal(LOCAL_UPNP)), AddPortMapping of the P2P port to this host every 20 minutes,
             DeletePortMapping when the node stops

The mapping thread starts when the node listens with `-upnp=1` (off by default, as a reference
build without miniupnpc). NODEXA_UPNP_SSDP=host:port sends the M-SEARCH to that address instead of
the multicast group (tests answer it with a local IGD).
"""
from __future__ import annotations

import os
import socket
import threading
import urllib.error
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET
from xml.sax.saxutils import escape

from ..utils import log

SSDP_ADDR = ("239.255.255.250", 1900)
IGD_SEARCH = ("urn:schemas-upnp-org:device:InternetGatewayDevice:1",
              "urn:schemas-upnp-org:device:InternetGatewayDevice:2")
WAN_SERVICES = ("urn:schemas-upnp-org:service:WANIPConnection:2", "urn:schemas-upnp-org:service:WANIPConnection:1",
                "urn:schemas-upnp-org:service:WANPPPConnection:1")
MAX_XML = 256 << 10  # a device description or SOAP reply larger than this is refused (LAN input)
LOCAL_UPNP = 3  # the reference's address score of a UPnP-discovered address (net.h LOCAL_UPNP)
REFRESH_S = 20 * 60  # AddPortMapping again every 20 minutes, as the reference
_SOAP_ENV = ("<?xml version=\"1.0\"?><s:Envelope xmlns:s=\"http://schemas.xmlsoap.org/soap/envelope/\" "
             "s:encodingStyle=\"http://schemas.xmlsoap.org/soap/encoding/\"><s:Body>{body}</s:Body></s:Envelope>")


class UPnPError(Exception):
    def __init__(self, msg: str, code: int = -1):
        super().__init__(msg)
        self.code = code


def _ssdp_target() -> tuple[str, int]:
    env = os.environ.get("NODEXA_UPNP_SSDP")
    if env:
        host, _, port = env.rpartition(":")
        return host, int(port)
    return SSDP_ADDR


def discover(timeout: float = 2.0, target: tuple[str, int] | None = None) -> list[str]:
    """upnpDiscover: the LOCATION URLs of the IGDs that answer an M-SEARCH within `timeout`."""
    target = target or _ssdp_target()
    found: list[str] = []
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM, socket.IPPROTO_UDP)
    try:
        s.setsockopt(socket.IPPROTO_IP, socket.IP_MULTICAST_TTL, 2)
        s.settimeout(timeout)
        for st in IGD_SEARCH:
            msg = (f"M-SEARCH * HTTP/1.1\r\nHOST: {SSDP_ADDR[0]}:{SSDP_ADDR[1]}\r\nST: {st}\r\n"
                   f"MAN: \"ssdp:discover\"\r\nMX: {max(1, int(timeout))}\r\n\r\n")
            try:
                s.sendto(msg.encode(), target)
            except OSError as e:
                raise UPnPError(f"M-SEARCH: {e}") from e
        while True:
            try:
                data, _ = s.recvfrom(4096)
            except (socket.timeout, OSError):
                break
            for line in data.decode(errors="replace").split("\r\n"):
                k, _, v = line.partition(":")
                if k.strip().lower() == "location" and v.strip() and v.strip() not in found:
                    found.append(v.strip())
    finally:
        s.close()
    return found


def _bounded(resp) -> bytes:
    data = resp.read(MAX_XML + 1)
    if len(data) > MAX_XML:
        raise UPnPError(f"reply larger than {MAX_XML} bytes")
    return data


def _local(tag: str) -> str:
    return tag.rsplit("}", 1)[-1]


def _http_url(url: str) -> str:
    """A URL an SSDP answer or a device description handed us, refused unless it is plain http
    (any LAN host can answer an M-SEARCH: no file:, ftp: or other scheme is ever opened)."""
    u = urllib.parse.urlparse(url)
    if u.scheme != "http" or not u.hostname:
        raise UPnPError(f"refusing non-http UPnP URL {url[:120]!r}")
    return url


def describe(location: str, timeout: float = 5.0) -> tuple[str, str, str]:
    """UPNP_GetValidIGD for one device: (control URL, service type, LAN address of this host)."""
    with urllib.request.urlopen(_http_url(location), timeout=timeout) as r:
        root = ET.fromstring(_bounded(r))
    base = next((e.text for e in root.iter() if _local(e.tag) == "URLBase" and e.text), location)
    services = [e for e in root.iter() if _local(e.tag) == "service"]
    for want in WAN_SERVICES:
        for svc in services:
            fields = {_local(c.tag): (c.text or "").strip() for c in svc}
            if fields.get("serviceType") == want and fields.get("controlURL"):
                control = _http_url(urllib.parse.urljoin(base, fields["controlURL"]))
                u = urllib.parse.urlparse(control)
                with socket.create_connection((u.hostname, u.port or 80), timeout=timeout) as c:
                    lan = c.getsockname()[0]
                return control, want, lan
    raise UPnPError("no WANIPConnection / WANPPPConnection service in the device description")


def soap(control: str, service: str, action: str, args: dict | None = None, timeout: float = 5.0) -> dict:
    """One SOAP action; the response's out-arguments, or UPnPError with the device's errorCode."""
    inner = "".join(f"<{k}>{escape(str(v))}</{k}>" for k, v in (args or {}).items())
    body = _SOAP_ENV.format(body=f"<u:{action} xmlns:u=\"{service}\">{inner}</u:{action}>").encode()
    req = urllib.request.Request(control, data=body, method="POST", headers={
        "Content-Type": "text/xml; charset=\"utf-8\"", "SOAPAction": f"\"{service}#{action}\""})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            root = ET.fromstring(_bounded(r))
    except urllib.error.HTTPError as e:
        try:
            root = ET.fromstring(_bounded(e))
        except ET.ParseError:
            raise UPnPError(f"{action}: HTTP {e.code}", e.code) from e
        code = next((el.text for el in root.iter() if _local(el.tag) == "errorCode"), None)
        desc = next((el.text for el in root.iter() if _local(el.tag) == "errorDescription"), "")
        raise UPnPError(f"{action}: {code} {desc}".strip(), int(code) if code and code.isdigit() else e.code) from e
    except OSError as e:
        raise UPnPError(f"{action}: {e}") from e
    resp = next((el for el in root.iter() if _local(el.tag) == action + "Response"), None)
    return {} if resp is None else {_local(c.tag): (c.text or "") for c in resp}


class PortMapper:
    """ThreadMapPort: discover an IGD, advertise its external address, map the P2P port (TCP, the
    same port outside and in) to this host and refresh the mapping every 20 minutes; stop() deletes
    it (the reference's thread interruption path)."""

    def __init__(self, port: int, add_local=None, discover_external: bool = True, description: str = "",
                 refresh_s: float = REFRESH_S, timeout: float = 2.0):
        self.port = int(port)
        self.add_local = add_local
        self.discover_external = discover_external
        from . import protocol

        self.description = description or "Clore " + protocol.USER_AGENT.strip("/")
        self.refresh_s = refresh_s
        self.timeout = timeout
        self.control = self.service = self.lan = None
        self.external_ip: str | None = None
        self.mapped = 0  # successful AddPortMapping calls
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def start(self) -> None:
        self._thread = threading.Thread(target=self._run, name="upnp", daemon=True)
        self._thread.start()

    def _run(self) -> None:
        try:
            locations = discover(self.timeout)
            for loc in locations:
                try:
                    self.control, self.service, self.lan = describe(loc)
                    break
                except (UPnPError, OSError, ET.ParseError, ValueError) as e:
                    log.log_printf(f"UPnP: {loc}: {e}")
            if self.control is None:
                log.log_printf("No valid UPnP IGDs found")
                return
            if self.discover_external:
                try:
                    ip = soap(self.control, self.service, "GetExternalIPAddress").get("NewExternalIPAddress", "")
                    if ip:
                        socket.inet_aton(ip)
                        self.external_ip = ip
                        log.log_printf(f"UPnP: ExternalIPAddress = {ip}")
                        if self.add_local is not None:
                            self.add_local(ip, self.port, LOCAL_UPNP)
                    else:
                        log.log_printf("UPnP: GetExternalIPAddress failed.")
                except (UPnPError, OSError) as e:
                    log.log_printf(f"UPnP: GetExternalIPAddress() returned {e}")
            while not self._stop.is_set():
                try:
                    soap(self.control, self.service, "AddPortMapping", {
                        "NewRemoteHost": "", "NewExternalPort": self.port, "NewProtocol": "TCP",
                        "NewInternalPort": self.port, "NewInternalClient": self.lan, "NewEnabled": 1,
                        "NewPortMappingDescription": self.description, "NewLeaseDuration": 0})
                    self.mapped += 1
                    log.log_printf("UPnP Port Mapping successful.")
                except UPnPError as e:
                    log.log_printf(f"AddPortMapping({self.port}, {self.port}, {self.lan}) failed with code {e.code} ({e})")
                self._stop.wait(self.refresh_s)
        except UPnPError as e:
            log.log_printf(f"UPnP: {e}")

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
        if self.control is not None and self.mapped:
            try:
                soap(self.control, self.service, "DeletePortMapping",
                     {"NewRemoteHost": "", "NewExternalPort": self.port, "NewProtocol": "TCP"})
                log.log_printf("UPNP_DeletePortMapping() returned: 0")
            except UPnPError as e:
                log.log_printf(f"UPNP_DeletePortMapping() returned: {e.code}")

"""UPnP port mapping (net/upnp.py, the reference's ThreadMapPort) against a local Internet Gateway
Device: an SSDP responder on a loopback UDP port (NODEXA_UPNP_SSDP points the M-SEARCH at it), a
device description with a WANIPConnection service nested in the device tree, and a SOAP control
endpoint that records every action and answers like a router."""
import http.server
import os
import socket
import threading
import time

import pytest

EXTERNAL_IP = "203.0.113.7"
DESC = """<?xml version="1.0"?>
<root xmlns="urn:schemas-upnp-org:device-1-0"><specVersion><major>1</major><minor>0</minor></specVersion>
<device><deviceType>urn:schemas-upnp-org:device:InternetGatewayDevice:1</deviceType>
 <deviceList><device><deviceType>urn:schemas-upnp-org:device:WANDevice:1</deviceType>
  <deviceList><device><deviceType>urn:schemas-upnp-org:device:WANConnectionDevice:1</deviceType>
   <serviceList><service><serviceType>urn:schemas-upnp-org:service:WANIPConnection:1</serviceType>
    <serviceId>urn:upnp-org:serviceId:WANIPConn1</serviceId><controlURL>/ctl/IPConn</controlURL>
    <eventSubURL>/evt/IPConn</eventSubURL><SCPDURL>/WANIPCn.xml</SCPDURL></service></serviceList>
  </device></deviceList></device></deviceList></device></root>"""


class FakeIGD:
    def __init__(self, fail_add: bool = False):
        self.actions: list[tuple[str, str]] = []
        self.fail_add = fail_add
        igd = self

        class H(http.server.BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                body = DESC.encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/xml")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_POST(self):
                n = int(self.headers.get("Content-Length", "0"))
                req = self.rfile.read(n).decode()
                action = self.headers.get("SOAPAction", "").strip('"').split("#")[-1]
                igd.actions.append((action, req))
                svc = "urn:schemas-upnp-org:service:WANIPConnection:1"
                if action == "AddPortMapping" and igd.fail_add:
                    body = ("<s:Envelope xmlns:s=\"http://schemas.xmlsoap.org/soap/envelope/\"><s:Body><s:Fault>"
                            "<detail><UPnPError xmlns=\"urn:schemas-upnp-org:control-1-0\"><errorCode>718</errorCode>"
                            "<errorDescription>ConflictInMappingEntry</errorDescription></UPnPError></detail>"
                            "</s:Fault></s:Body></s:Envelope>").encode()
                    self.send_response(500)
                else:
                    out = f"<NewExternalIPAddress>{EXTERNAL_IP}</NewExternalIPAddress>" \
                        if action == "GetExternalIPAddress" else ""
                    body = (f"<s:Envelope xmlns:s=\"http://schemas.xmlsoap.org/soap/envelope/\"><s:Body>"
                            f"<u:{action}Response xmlns:u=\"{svc}\">{out}</u:{action}Response></s:Body>"
                            f"</s:Envelope>").encode()
                    self.send_response(200)
                self.send_header("Content-Type", "text/xml")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.http = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.udp = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.udp.bind(("127.0.0.1", 0))
        self.udp.settimeout(0.2)
        self.searches: list[str] = []
        self._stop = threading.Event()
        threading.Thread(target=self.http.serve_forever, daemon=True).start()
        threading.Thread(target=self._ssdp, daemon=True).start()

    @property
    def ssdp(self) -> str:
        return "127.0.0.1:%d" % self.udp.getsockname()[1]

    def _ssdp(self):
        while not self._stop.is_set():
            try:
                data, addr = self.udp.recvfrom(2048)
            except OSError:
                continue
            msg = data.decode()
            self.searches.append(msg)
            if msg.startswith("M-SEARCH") and "InternetGatewayDevice" in msg:
                loc = "http://127.0.0.1:%d/rootDesc.xml" % self.http.server_address[1]
                self.udp.sendto(("HTTP/1.1 200 OK\r\nCACHE-CONTROL: max-age=120\r\nST: "
                                 "urn:schemas-upnp-org:device:InternetGatewayDevice:1\r\nUSN: uuid:fake::igd\r\n"
                                 f"LOCATION: {loc}\r\n\r\n").encode(), addr)

    def close(self):
        self._stop.set()
        self.http.shutdown()
        self.udp.close()


@pytest.fixture()
def igd(monkeypatch):
    g = FakeIGD()
    monkeypatch.setenv("NODEXA_UPNP_SSDP", g.ssdp)
    yield g
    g.close()


def _wait(cond, t=10.0):
    end = time.time() + t
    while time.time() < end:
        if cond():
            return True
        time.sleep(0.05)
    return False


def test_discover_describe_and_control(igd):
    from nodexa_chain_core_amd.net import upnp

    locs = upnp.discover(0.5)
    assert len(locs) == 1 and locs[0].endswith("/rootDesc.xml")
    assert all("MAN: \"ssdp:discover\"" in m for m in igd.searches)
    control, service, lan = upnp.describe(locs[0])
    assert control.endswith("/ctl/IPConn") and service.endswith("WANIPConnection:1") and lan == "127.0.0.1"
    assert upnp.soap(control, service, "GetExternalIPAddress") == {"NewExternalIPAddress": EXTERNAL_IP}


def test_port_mapper_maps_advertises_refreshes_and_deletes(igd):
    from nodexa_chain_core_amd.net.upnp import LOCAL_UPNP, PortMapper

    local = []
    m = PortMapper(18444, add_local=lambda h, p, s: local.append((h, p, s)), refresh_s=0.2, timeout=0.5)
    m.start()
    assert _wait(lambda: m.mapped >= 2)  # mapped, then refreshed
    assert local == [(EXTERNAL_IP, 18444, LOCAL_UPNP)]
    adds = [body for a, body in igd.actions if a == "AddPortMapping"]
    assert "<NewExternalPort>18444</NewExternalPort>" in adds[0] and "<NewInternalPort>18444</NewInternalPort>" in adds[0]
    assert "<NewProtocol>TCP</NewProtocol>" in adds[0] and "<NewInternalClient>127.0.0.1</NewInternalClient>" in adds[0]
    assert "<NewPortMappingDescription>Clore " in adds[0]
    m.stop()
    assert igd.actions[-1][0] == "DeletePortMapping" and "<NewExternalPort>18444</NewExternalPort>" in igd.actions[-1][1]


def test_port_mapper_survives_refusal_and_absence(monkeypatch):
    from nodexa_chain_core_amd.net.upnp import PortMapper

    g = FakeIGD(fail_add=True)  # the router refuses the mapping (718): logged, retried, nothing to delete
    monkeypatch.setenv("NODEXA_UPNP_SSDP", g.ssdp)
    try:
        m = PortMapper(18445, refresh_s=0.1, timeout=0.5)
        m.start()
        assert _wait(lambda: sum(a == "AddPortMapping" for a, _ in g.actions) >= 2)
        m.stop()
        assert m.mapped == 0 and not any(a == "DeletePortMapping" for a, _ in g.actions)
    finally:
        g.close()
    with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:  # nobody answers: no IGD, no mapping
        s.bind(("127.0.0.1", 0))
        monkeypatch.setenv("NODEXA_UPNP_SSDP", "127.0.0.1:%d" % s.getsockname()[1])
        m = PortMapper(18446, timeout=0.3)
        m.start()
        m._thread.join(5)
        assert m.control is None and m.mapped == 0


def test_node_upnp_flag(core, tmp_path, igd):
    """-upnp=1 on a listening node: the external address shows up in getnetworkinfo's localaddresses."""
    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.rpc.client import RPCClient
    from nodexa_chain_core_amd.utils.config import ArgsManager

    args = ArgsManager()
    args.parse_parameters(["-regtest", f"-datadir={tmp_path}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
                           "-printtoconsole=0", "-listen", "-port=0", "-upnp=1", "-listenonion=0"])
    n = Node(args)
    n.start()
    try:
        c = RPCClient("127.0.0.1", n.rpc.port, "u", "p")
        assert _wait(lambda: any(x["address"] == EXTERNAL_IP for x in c.getnetworkinfo()["localaddresses"]))
        assert n.upnp.mapped >= 1
    finally:
        n.stop()
    assert igd.actions[-1][0] == "DeletePortMapping"


def test_non_http_locations_are_refused(tmp_path):
    """Any LAN host can answer an M-SEARCH: a file: (or other non-http) LOCATION or controlURL is
    never opened."""
    from nodexa_chain_core_amd.net import upnp

    f = tmp_path / "desc.xml"
    f.write_text(DESC)
    with pytest.raises(upnp.UPnPError, match="non-http"):
        upnp.describe(f.as_uri())
    g = FakeIGD()
    try:
        bad = DESC.replace("<controlURL>/ctl/IPConn</controlURL>", "<controlURL>file:///etc/passwd</controlURL>")
        orig = g.http.RequestHandlerClass.do_GET

        def do_get(self):
            body = bad.encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        g.http.RequestHandlerClass.do_GET = do_get
        with pytest.raises(upnp.UPnPError, match="non-http"):
            upnp.describe("http://127.0.0.1:%d/rootDesc.xml" % g.http.server_address[1])
        g.http.RequestHandlerClass.do_GET = orig
    finally:
        g.close()

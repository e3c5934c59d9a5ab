"""Argument / config-file handling with the reference's ArgsManager semantics.

Parity: ArgsManager (src/util.h:225), ParseParameters (src/util.cpp:407) —
`-name`, `-name=value`, `--name=value`, `-noname` (negation), repeated
options become lists; ReadConfigFile (src/util.cpp:631) — `name=value`
lines, `#` comments, `[main]/[test]/[regtest]` sections that apply only to
that network; command line wins over the file; SoftSetArg / ForceSetArg;
network selection from -regtest / -testnet (SelectParams).

New engine flags: -gpus=0,1,.. -kawpowactivationtime= -equihash
-gpuintensity= -dagcache= -gpufailrate= -dropshare= -strictheight -dbformat=leveldb|journal
"""
from __future__ import annotations

import os
import threading

DEFAULT_CONF = "nodexa.conf"
NETWORKS = ("main", "test", "regtest")


class ArgsManager:
    def __init__(self) -> None:
        self._lock = threading.RLock()
        self._cli: dict[str, list[str]] = {}
        self._conf: dict[str, list[str]] = {}
        self._forced: dict[str, list[str]] = {}
        self._network = "main"

    # ------------------------------------------------------------ parsing
    @staticmethod
    def _norm(key: str) -> tuple[str, bool]:
        key = key.lstrip("-")
        if key.startswith("no") and len(key) > 2 and not key.startswith("nonce"):
            return key[2:], True
        return key, False

    def parse_parameters(self, argv: list[str]) -> list[str]:
        """Parse `-flag[=value]` options; returns the positional remainder."""
        rest: list[str] = []
        with self._lock:
            self._cli.clear()
            for i, a in enumerate(argv):
                if not a.startswith("-") or a in ("-", "--"):
                    rest.extend(argv[i:])
                    break
                name, _, value = a.partition("=")
                key, neg = self._norm(name)
                if neg:
                    value = "0" if value in ("", "1") else ("1" if value == "0" else value)
                elif "=" not in a:
                    value = "1"
                self._cli.setdefault(key, []).append(value)
            self._network = self._select_network()
        return rest

    def read_config_file(self, path: str) -> None:
        if not os.path.exists(path):
            return
        section = None
        with self._lock, open(path) as f:
            for raw in f:
                line = raw.split("#", 1)[0].strip()
                if not line:
                    continue
                if line.startswith("[") and line.endswith("]"):
                    section = line[1:-1].strip()
                    continue
                name, _, value = line.partition("=")
                key, neg = self._norm(name.strip())
                value = value.strip()
                if neg:
                    value = "0"
                elif "=" not in line:
                    value = "1"
                full = key if section is None else f"{section}.{key}"
                self._conf.setdefault(full, []).append(value)
            self._network = self._select_network()

    def _select_network(self) -> str:
        reg = self._raw_bool("regtest")
        test = self._raw_bool("testnet")
        if reg and test:
            raise ValueError("Invalid combination of -regtest and -testnet.")
        return "regtest" if reg else ("test" if test else "main")

    # ------------------------------------------------------------ getters
    def _values(self, key: str) -> list[str] | None:
        key = key.lstrip("-")
        with self._lock:
            if key in self._forced:
                return self._forced[key]
            if key in self._cli:
                return self._cli[key]
            sec = f"{self._network}.{key}"
            if sec in self._conf:
                return self._conf[sec]
            if key in self._conf:
                return self._conf[key]
        return None

    def _raw_bool(self, key: str) -> bool:
        v = self._cli.get(key) or self._conf.get(key)
        return bool(v) and _truthy(v[-1])

    @property
    def network(self) -> str:
        return self._network

    def is_set(self, key: str) -> bool:
        return self._values(key) is not None

    def get(self, key: str, default: str | None = None) -> str | None:
        v = self._values(key)
        return v[-1] if v else default

    def get_int(self, key: str, default: int) -> int:
        v = self.get(key)
        try:
            return int(v) if v is not None else default
        except ValueError:
            return default

    def get_bool(self, key: str, default: bool = False) -> bool:
        v = self.get(key)
        return default if v is None else _truthy(v)

    def get_list(self, key: str) -> list[str]:
        return list(self._values(key) or [])

    def soft_set(self, key: str, value: str) -> bool:
        """Set only if the user did not (SoftSetArg)."""
        if self.is_set(key):
            return False
        self.force_set(key, value)
        return True

    def force_set(self, key: str, value: str) -> None:
        with self._lock:
            self._forced[key.lstrip("-")] = [value]

    def data_dir(self) -> str:
        base = os.path.expanduser(self.get("datadir", os.path.join("~", ".nodexa")))
        path = base if self._network == "main" else os.path.join(base, "testnet7" if self._network == "test"
                                                                 else "regtest")
        os.makedirs(path, exist_ok=True)
        return path


def _truthy(v: str) -> bool:
    v = v.strip().lower()
    if v in ("", "1", "true", "yes", "on"):
        return True
    if v in ("0", "false", "no", "off"):
        return False
    try:
        return int(v) != 0
    except ValueError:
        return True


def gpu_list(args: ArgsManager) -> list[int]:
    """`-gpus=0,1,3` -> [0, 1, 3]; `-gpus=all` -> every visible device; unset -> []."""
    v = args.get("gpus")
    if v is None or v.strip().lower() in ("", "none", "off"):
        return []
    if v == "all":
        import torch

        return list(range(torch.cuda.device_count()))
    return [int(x) for x in v.split(",") if x.strip() != ""]


g_args = ArgsManager()

"""Shell notifications: -blocknotify, -walletnotify, -alertnotify.

Parity (behaviour): src/init.cpp BlockNotifyCallback (`-blocknotify=<cmd>`, "%s" replaced by the
new tip's block hash, run on each tip change outside initial download), src/wallet/wallet.cpp
AddToWallet (`-walletnotify=<cmd>`, "%s" = the txid, on every new or updated wallet transaction)
and src/validation.cpp AlertNotify (`-alertnotify=<cmd>`, "%s" = the message with quotes and
shell metacharacters stripped). Each command runs through the shell on its own detached thread,
as runCommand on boost::thread does, so a slow script never blocks validation.
"""
from __future__ import annotations

import re
import subprocess
import threading

from . import log

_SAFE = re.compile(r"[^A-Za-z0-9 .,;\-_/:?@]")


def run_command(cmd: str) -> threading.Thread:
    def _run():
        try:
            rc = subprocess.run(cmd, shell=True).returncode  # noqa: S602 — the operator's own command
        except OSError as e:
            log.log_printf(f"runCommand error: {e}")
            return
        if rc:
            log.log_printf(f"runCommand error: system({cmd}) returned {rc}")

    t = threading.Thread(target=_run, name="notify", daemon=True)
    t.start()
    return t


def substitute(template: str, value: str) -> str:
    return template.replace("%s", value)


def alert_text(msg: str) -> str:
    """AlertNotify's SanitizeString + single-quote wrapping of the message."""
    return "'" + _SAFE.sub("", msg) + "'"


class Notifier:
    """Holds the three templates; `None` disables a notification."""

    def __init__(self, block: str | None = None, wallet: str | None = None, alert: str | None = None):
        self.block, self.wallet, self.alert = block or None, wallet or None, alert or None

    def block_tip(self, block_hash_hex: str, initial_download: bool = False):
        if self.block and not initial_download:
            return run_command(substitute(self.block, block_hash_hex))
        return None

    def wallet_tx(self, txid_hex: str):
        if self.wallet:
            return run_command(substitute(self.wallet, txid_hex))
        return None

    def alert_msg(self, msg: str):
        if self.alert:
            return run_command(substitute(self.alert, alert_text(msg)))
        return None

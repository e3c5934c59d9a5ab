"""Key wallet (wallet.py) and its JSON-RPC methods (rpc/methods_wallet.py)."""
from .wallet import Wallet, WalletError

__all__ = ["Wallet", "WalletError"]

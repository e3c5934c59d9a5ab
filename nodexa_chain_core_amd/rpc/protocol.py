"""JSON-RPC protocol constants and helpers (src/rpc/protocol.h parity)."""
from __future__ import annotations

import contextvars

# the wallet a JSON-RPC request addresses: None outside a request, "" for the "/" endpoint, the
# name for "/wallet/<name>" (multiwallet endpoints, src/wallet/rpcwallet.cpp:40-53)
REQUEST_WALLET: contextvars.ContextVar = contextvars.ContextVar("request_wallet", default=None)

# RPCErrorCode values used by the reference (src/rpc/protocol.h)
RPC_INVALID_REQUEST = -32600
RPC_METHOD_NOT_FOUND = -32601
RPC_WALLET_NOT_FOUND = -18      # the /wallet/<name> endpoint names no loaded wallet
RPC_WALLET_NOT_SPECIFIED = -19  # several wallets loaded and the request named none
RPC_INVALID_PARAMS = -32602
RPC_INTERNAL_ERROR = -32603
RPC_PARSE_ERROR = -32700
RPC_MISC_ERROR = -1
RPC_FORBIDDEN_BY_SAFE_MODE = -2
RPC_WALLET_ERROR = -4
RPC_WALLET_INSUFFICIENT_FUNDS = -6
RPC_TYPE_ERROR = -3
RPC_INVALID_ADDRESS_OR_KEY = -5
RPC_OUT_OF_MEMORY = -7
RPC_INVALID_PARAMETER = -8
RPC_DATABASE_ERROR = -20
RPC_DESERIALIZATION_ERROR = -22
RPC_VERIFY_ERROR = -25
RPC_VERIFY_REJECTED = -26
RPC_VERIFY_ALREADY_IN_CHAIN = -27
RPC_TRANSACTION_ERROR = -25  # RPC_VERIFY_ERROR's alias for missing inputs (src/rpc/protocol.h)
RPC_IN_WARMUP = -28
RPC_METHOD_DEPRECATED = -32
RPC_CLIENT_NOT_CONNECTED = -9
RPC_CLIENT_IN_INITIAL_DOWNLOAD = -10


class RPCError(Exception):
    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code
        self.message = message

    def to_json(self) -> dict:
        return {"code": self.code, "message": self.message}


def http_status_for(code: int) -> int:
    """JSONErrorReply status mapping (src/httprpc.cpp)."""
    if code == RPC_INVALID_REQUEST:
        return 400
    if code == RPC_METHOD_NOT_FOUND:
        return 404
    return 500


def reply(result, error, id_) -> dict:
    return {"result": result, "error": error, "id": id_}

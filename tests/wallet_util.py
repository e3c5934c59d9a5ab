"""Test helpers: fund a node's wallet with mature coinbase outputs and build signed spends
through the node's own RPCs (createrawtransaction + signrawtransaction)."""


def fund(c, blocks: int = 101) -> str:
    """Mine `blocks` blocks to a fresh wallet address; with 101 the first coinbase is mature."""
    w = c.getnewaddress()
    c.generatetoaddress(blocks, w)
    return w


def spend(c, prev_txid: str, vout: int, prev_amount: float, to_addr: str, amount: float,
          fee: float = 0.01) -> str:
    """Signed raw tx paying `amount` to `to_addr` and the rest (minus `fee`) back to the wallet."""
    outs = {to_addr: amount}
    change = round(prev_amount - amount - fee, 8)
    if change > 0:
        outs[c.getnewaddress()] = change
    raw = c.createrawtransaction([{"txid": prev_txid, "vout": vout}], outs)
    signed = c.signrawtransaction(raw)
    assert signed["complete"], signed
    return signed["hex"]


def mature_coin(c) -> dict:
    coins = [u for u in c.listunspent() if u["spendable"]]
    assert coins, "no mature wallet output"
    return max(coins, key=lambda u: u["amount"])

"""nodexad — the engine daemon (AppInit / AppInitMain / Shutdown equivalent).

Parity: main -> AppInit (src/clore_blockchaind.cpp:66-198) -> AppInitMain
(src/init.cpp:1322-1966): parse args + config file, select network, lock the
data directory, load the block index (here: rebuild from blk files), start the
RPC server (warm-up until the chain is loaded), start the miner when -gen,
wait for shutdown; Interrupt/Shutdown (src/init.cpp:172,355).

MI355X specifics: `-gpus=0,1,...` selects the devices the miner and the batch
verifier use (one DAG per device, built on the GPU); `-kawpowactivationtime=<t>`
overrides the KawPow activation time. Every network's default is the reference's
(regtest: 3582830167, src/chainparams.cpp:566-570, so a default regtest node mines
80-byte X16RV2 headers exactly as clore_blockchaind does);
`-kawpowactivationtime=1524179367` (genesis + 1) makes every mined regtest block
KawPow. `-equihash=<time>` enables the Equihash(200,9) extension from that time
(off by default).

    python -m nodexa_chain_core_amd.node -regtest -rpcport=19443 -miningaddress=<addr> [-gpus=0]
        [-kawpowactivationtime=1524179367]
"""
from __future__ import annotations

import fcntl
import os
import signal
import sys
import threading
import time

from . import core
from .chain.state import ChainState, make_params
from .miner.assembler import BlockAssembler, ExtraNonce
from .miner.service import Miner
from .rpc import (methods, methods_assets, methods_ext, methods_index, methods_messages, methods_util, methods_wallet,
                  methods_wallet_ext)
from .rpc.server import RPCServer, RPCTable, delete_cookie, make_cookie
from .utils import log, metrics
from .utils.config import ArgsManager, gpu_list

_core = core()


# chainparams vSeeds (src/chainparams.cpp:184-186, 346): DNS names resolved by ThreadDNSAddressSeed
DNS_SEEDS = {"main": ["seed.clore.ai", "seed1.clore.ai", "seed2.clore.ai"], "test": ["testnet.clore.ai"], "regtest": []}


DEFAULT_WALLET = "wallet.json"  # -wallet default (the reference: wallet.dat)

class Node:
    def __init__(self, args: ArgsManager):
        self.args = args
        self.network = args.network
        act = args.get("kawpowactivationtime")
        eq = args.get("equihash")
        self.params = make_params(self.network, int(act) if act is not None else None,
                                  int(eq) if eq not in (None, "", "1") else None)
        if not args.get_bool("checkpoints", True):  # -checkpoints=0: fCheckpointsEnabled = false
            self.params.clear_checkpoints()
        self.datadir = args.data_dir() if args.get("datadir") is not None or not args.get_bool("nodatadir") else None
        self._lock_file = None
        self._shutdown = threading.Event()
        self.last_block_tx = 0
        self.last_block_weight = 0
        self.pprpc_templates: dict[str, object] = {}
        self.equihash_templates: dict[str, object] = {}
        self._last_pprpc: tuple[str, float] | None = None
        self.gpus = gpu_list(args)
        self.rpc_witness = True  # -rpcserialversion=1
        self.asset_index = args.get_bool("assetindex", False)  # -assetindex: per-address asset balance RPCs
        self.state: ChainState | None = None
        self.miner: Miner | None = None
        self.rpc: RPCServer | None = None
        self.table = RPCTable()
        addr = args.get("miningaddress")
        self.mining_script = None
        if addr:
            self.mining_script = _core.address_to_script(addr, self.params.pubkey_prefix, self.params.script_prefix)
            if self.mining_script is None:
                raise SystemExit(f"Error: invalid -miningaddress {addr} for {self.network}")

    # ------------------------------------------------------------------ lifecycle
    def lock_datadir(self) -> None:
        if self.datadir is None:
            return
        path = os.path.join(self.datadir, ".lock")
        self._lock_file = open(path, "a+")
        try:
            fcntl.flock(self._lock_file, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            raise SystemExit(f"Cannot obtain a lock on data directory {self.datadir}. Nodexa is probably already running.")

    def _check_legacy_flags(self) -> None:
        """AppInitParameterInteraction's removed / renamed options: hard errors for -socks,
        -rpcssl and -tor, warnings for options that are ignored now."""
        a = self.args
        if a.is_set("socks"):
            raise SystemExit("Unsupported argument -socks found. Setting SOCKS version isn't possible anymore, "
                             "only SOCKS5 proxies are supported.")
        if a.get_bool("rpcssl", False):
            raise SystemExit("SSL mode for RPC (-rpcssl) is no longer supported.")
        if a.is_set("tor"):
            raise SystemExit("Unsupported argument -tor found, use -onion.")
        for old, hint in (("benchmark", "-benchmark is ignored, use -debug=bench."),
                          ("debugnet", "Unsupported argument -debugnet ignored, use -debug=net."),
                          ("whitelistalwaysrelay", "Unsupported argument -whitelistalwaysrelay ignored, use "
                                                   "-whitelistrelay and/or -whitelistforcerelay."),
                          ("blockminsize", "Unsupported argument -blockminsize ignored.")):
            if a.is_set(old):
                log.log_printf("Warning: " + hint)

    def start(self) -> None:
        """AppInit: on a start-up error the node shuts down what it had brought up (RPC server,
        chain state, data-directory lock) before the error propagates, as the reference's
        Shutdown() after a failed AppInitMain."""
        try:
            self._start()
        except BaseException:
            try:
                self.stop()
            except Exception as e:  # noqa: BLE001 — the start-up error is the one to report
                log.log_printf(f"shutdown after a failed start: {e}")
            raise

    def _start(self) -> None:
        a = self.args
        if not a.get_bool("sysperms", False):
            os.umask(0o077)  # files this node creates are private unless -sysperms (src/init.cpp)
        self._check_legacy_flags()
        log.configure(a.get_list("debug"), a.get_list("debugexclude"),
                      os.path.join(self.datadir, "debug.log") if self.datadir else None,
                      console=a.get_bool("printtoconsole", True), timestamps=a.get_bool("logtimestamps", True),
                      micros=a.get_bool("logtimemicros", False), ips=a.get_bool("logips", False),
                      shrink=a.get_bool("shrinkdebugfile") if a.is_set("shrinkdebugfile") else None)
        self.lock_datadir()
        self._pidfile = None
        if self.datadir is not None:  # CreatePidFile: -pid=<file> (relative to the data directory)
            self._pidfile = os.path.join(self.datadir, a.get("pid", "nodexad.pid"))
            with open(self._pidfile, "w") as f:
                f.write(f"{os.getpid()}\n")
        # RPC comes up first in warm-up mode (AppInitServers)
        self.table.warmup = "Loading block index..."
        self.table.safe_mode = self.observe_safe_mode
        methods.register(self.table, self)
        methods_ext.register(self.table, self)
        if a.get_bool("server", True):
            self._start_rpc()
        dagcache = a.get("dagcache")
        if dagcache:  # on-disk light caches keyed by epoch seed (SURVEY §5 checkpoint/resume)
            if dagcache == "1":
                dagcache = os.path.join(self.datadir or ".", "dagcache")
            os.makedirs(dagcache, exist_ok=True)
            _core.set_light_cache_dir(dagcache)
        if a.get_bool("debuglockorder", False):  # DEBUG_LOCKORDER (src/sync.cpp) for the Python-side locks
            from .utils import sync

            sync.enable(True)
        indexes = {k: a.get_bool(k, False) for k in ("txindex", "addressindex", "spentindex", "timestampindex")}
        self.state = ChainState(self.params, self.datadir, strict_height=a.get_bool("strictheight", False),
                                reindex=a.get_bool("reindex", False), indexes=indexes,
                                db_format=a.get("dbformat") or None,  # -dbformat=leveldb|journal
                                reindex_chainstate=a.get_bool("reindex-chainstate", False))
        for flag, attr in (("maxreorg", "max_reorg_depth"), ("minreorgpeers", "min_reorg_peers"),
                           ("minreorgage", "min_reorg_age")):  # reorg guard knobs (src/init.cpp)
            if a.is_set(flag):
                setattr(self.params, attr, a.get_int(flag, getattr(self.params, attr)))
        if self.network == "regtest" and a.is_set("blockversion"):  # -blockversion (src/miner.cpp:146-149)
            self.state.block_version_override = a.get_int("blockversion", 0)
        self.wallets: dict = {}  # name -> Wallet, in -wallet order (the first is the default)
        if not a.get_bool("disablewallet", False):  # -disablewallet (src/wallet/init.cpp)
            from .wallet import Wallet

            from .wallet.history import WalletHistory

            from .rpc.protocol import REQUEST_WALLET

            names = a.get_list("wallet") or [DEFAULT_WALLET]
            for k, name in enumerate(names):  # WalletVerify (src/wallet/init.cpp): plain, distinct file names
                if os.path.basename(name) != name or name in (".", ".."):
                    raise SystemExit(f"Error loading wallet {name}. -wallet parameter must only specify a filename (not a path).")
                if name in names[:k]:
                    raise SystemExit(f"Error loading wallet {name}. Duplicate -wallet filename specified.")
            for name in names:
                wpath, hist_path = self._wallet_paths(name)
                # -bip44 (default on): a new wallet derives from BIP39 words (-mnemonic /
                # -mnemonicpassphrase; the default wallet only)
                first = not self.wallets
                dat = self._reference_wallet_file(name, wpath)
                w = Wallet(self.state, self.params, wpath, bip44=a.get_bool("bip44", True),
                           mnemonic=(a.get("mnemonic", "") or "") if first else "",
                           mnemonic_passphrase=(a.get("mnemonicpassphrase", "") or "") if first else "",
                           import_from=dat, keep_uncompressed=a.get_bool("walletkeepuncompressed", False))
                if w.import_report is not None:
                    log.log_printf(f"Imported reference wallet {dat} into {wpath}: {w.import_report}")
                w.name = name
                self.wallets[name] = w
                rescan = hist_path is not None and not os.path.exists(hist_path) and bool(w.keys)
                rescan = rescan or a.get_bool("rescan", False)  # -rescan: rebuild the history at start-up
                w.history = WalletHistory(w, hist_path)
                token = REQUEST_WALLET.set(name)  # rescans below address this wallet
                try:
                    zap = a.get_int("zapwallettxes", 0)
                    if zap:  # -zapwallettxes=1|2: drop every wallet transaction, rescan (1 keeps their metadata)
                        hist = w.history
                        keep = {t: (x.comment, x.comment_to, x.from_account) for t, x in hist.txs.items()} if zap == 1 else {}
                        hist.txs.clear()
                        methods_wallet.rescan(self)
                        for t, (cm, ct, acct) in keep.items():
                            x = hist.txs.get(t)
                            if x is not None:
                                x.comment, x.comment_to, x.from_account = cm, ct, acct
                        hist.save()
                        log.log_printf(f"Zapped wallet transactions (mode {zap}); {len(hist.txs)} found again by the rescan")
                    elif rescan:
                        methods_wallet.rescan(self)
                finally:
                    REQUEST_WALLET.reset(token)
                self.state.register(w.history)
            methods_wallet.register(self.table, self)
            methods_wallet_ext.register(self.table, self)
        self._asset_wallets: dict = {}  # wallet name -> AssetWallet, built on first use
        from .wallet.messages import MessageStore
        from .wallet.rewards import MINIMUM_REWARDS_PAYOUT_HEIGHT, Rewards

        # asset messaging (-disablemessaging) and reward snapshots (-minrewardheight)
        self.messages = MessageStore(self.state, self.wallet,
                                     os.path.join(self.datadir, "messages.json") if self.datadir else None,
                                     enabled=not a.get_bool("disablemessaging", False))
        self.state.register(self.messages)
        self.rewards = Rewards(self.state, self.wallet, self.asset_wallet_instance,
                               os.path.join(self.datadir, "rewards.json") if self.datadir else None,
                               a.get_int("minrewardheight", MINIMUM_REWARDS_PAYOUT_HEIGHT))
        self.state.register(self.rewards)
        methods_assets.register(self.table, self)  # chain-state asset methods work without a wallet
        methods_messages.register(self.table, self)
        methods_index.register(self.table, self)
        methods_util.register(self.table, self)
        if a.get("minrelaytxfee") is not None:  # -minrelaytxfee=<CLORE per kvB>
            self.state.min_relay_fee = round(float(a.get("minrelaytxfee")) * 100_000_000)
        if a.get("incrementalrelayfee") is not None:
            self.state.incremental_relay_fee = round(float(a.get("incrementalrelayfee")) * 100_000_000)
        self.state.enable_replacement = a.get_bool("mempoolreplacement", self.state.enable_replacement)
        st, coin = self.state, 100_000_000  # relay / package / block policy knobs (src/init.cpp)
        av = a.get("assumevalid", self.params_assume_valid())  # -assumevalid=<hex>; 0 = check every script
        st.assume_valid = None if av in (None, "", "0") else bytes.fromhex(av.rjust(64, "0"))[::-1]
        if a.get("minimumchainwork"):
            st.minimum_chain_work = int(a.get("minimumchainwork"), 16)
        st.max_tip_age = a.get_int("maxtipage", st.max_tip_age)
        st.db_crash_ratio = a.get_int("dbcrashratio", 0)
        st.bytes_per_sigop = a.get_int("bytespersigop", st.bytes_per_sigop)
        st.print_priority = a.get_bool("printpriority", False)
        self._configure_pruning(a)
        # -dbcache (MiB, src/txdb.h nDefaultDbCache / nMinDbCache / nMaxDbCache): bounds the UTXO
        # changes held between flushes; a flush also runs every flush_interval blocks
        st.coins_cache_bytes = min(max(a.get_int("dbcache", 450), 4), 16384) << 20
        # -checkblockindex: off by default here (the reference turns it on for regtest; it is an
        # O(chain) walk per block, so the suites enable it where they test it)
        st.check_block_index_enabled = a.get_bool("checkblockindex", False)
        ser = a.get_int("rpcserialversion", 1)  # -rpcserialversion: 0 = non-segwit, 1 = segwit serialization
        if ser not in (0, 1):
            raise SystemExit("unknown rpcserialversion requested." if ser > 1 else "rpcserialversion must be non-negative.")
        self.rpc_witness = ser == 1
        if a.is_set("mocktime"):  # -mocktime=<n> (regtest tooling): SetMockTime at start-up
            if self.network != "regtest":
                raise SystemExit("-mocktime is for regression testing (-regtest mode) only")
            st.mocktime = a.get_int("mocktime", 0)
        for spec in a.get_list("vbparams"):  # -vbparams=deployment:start:end (regtest only)
            self._apply_vbparams(spec)
        self._verify_db(a.get_int("checkblocks", 6), a.get_int("checklevel", 3))
        st.datacarrier = a.get_bool("datacarrier", True)
        st.datacarrier_size = a.get_int("datacarriersize", st.datacarrier_size)
        st.permit_bare_multisig = a.get_bool("permitbaremultisig", True)
        if a.get("dustrelayfee") is not None:
            st.dust_relay_fee = round(float(a.get("dustrelayfee")) * coin)
        st.ancestor_limits = (a.get_int("limitancestorcount", st.ancestor_limits[0]),
                              a.get_int("limitancestorsize", st.ancestor_limits[1] // 1000) * 1000)
        st.descendant_limits = (a.get_int("limitdescendantcount", st.descendant_limits[0]),
                                a.get_int("limitdescendantsize", st.descendant_limits[1] // 1000) * 1000)
        max_pool = a.get_int("maxmempool", st.max_mempool_bytes // 1_000_000)
        min_pool = st.descendant_limits[1] * 40 // 1_000_000  # nMempoolSizeMin = limitdescendantsize * 40
        if max_pool < min_pool:
            raise SystemExit(f"-maxmempool must be at least {min_pool} MB")
        st.max_mempool_bytes = max_pool * 1_000_000
        st.mempool_expiry = a.get_int("mempoolexpiry", st.mempool_expiry // 3600) * 3600
        if a.get("maxtxfee") is not None:
            st.max_tx_fee = round(float(a.get("maxtxfee")) * coin)
        st.block_max_weight = a.get_int("blockmaxweight", st.block_max_weight)
        if a.is_set("blockmaxsize"):
            st.block_max_size = a.get_int("blockmaxsize", 0)
        if a.get("blockmintxfee") is not None:
            st.block_min_fee_rate = round(float(a.get("blockmintxfee")) * coin)
        self.state.require_standard = not a.get_bool("acceptnonstdtxn", not self.state.require_standard)
        for w in self.wallets.values():  # -paytxfee / -fallbackfee / -txconfirmtarget (amounts in CLORE per kB)
            w.walletrbf = a.get_bool("walletrbf", False)
            if a.get("paytxfee") is not None:
                w.pay_tx_fee = round(float(a.get("paytxfee")) * 100_000_000)
            if a.get("fallbackfee") is not None:
                w.fallback_fee = round(float(a.get("fallbackfee")) * 100_000_000)
            w.tx_confirm_target = a.get_int("txconfirmtarget", w.tx_confirm_target)
            if a.get("mintxfee") is not None:
                w.min_tx_fee = round(float(a.get("mintxfee")) * 100_000_000)
            w.keypool_size = max(1, a.get_int("keypool", w.keypool_size))
            w.broadcast = a.get_bool("walletbroadcast", True)
            w.spend_zeroconf_change = a.get_bool("spendzeroconfchange", True)
            if a.get("discardfee") is not None:
                w.discard_fee = round(float(a.get("discardfee")) * 100_000_000)
            w.reject_long_chains = a.get_bool("walletrejectlongchains", False)
        # Berkeley DB tuning / recovery options of the reference wallet (src/wallet/init.cpp): the
        # wallet here is a JSON file rewritten atomically on every change (older layouts upgraded
        # on load), so these have nothing to act on
        for flag in ("dblogsize", "flushwallet", "privdb", "salvagewallet", "upgradewallet", "fuzzmessagestest"):
            if a.is_set(flag):
                log.log_printf(f"-{flag} has no effect in this build")
        # -maxsigcachesize (MiB, src/script/sigcache.cpp InitSignatureCache): bounded by its 32-byte entries
        _core.sigcache_set_max_bytes(max(0, a.get_int("maxsigcachesize", 32)) << 20)
        par = int(a.get("par", "0"))  # -par: 0 = one per core (as the reference), <0 leaves that many cores free
        cores = os.cpu_count() or 1
        self.state.script_threads = max(1, min(16, cores + par if par <= 0 else par))
        self.state.gpu_signatures = a.get("gpusigs", "auto")  # -gpusigs=auto|on|off: GPU batch ECDSA in blocks
        if self.datadir is not None:  # fee_estimates.dat (src/init.cpp: est_filein), before the mempool
            self.state.load_fee_estimates(os.path.join(self.datadir, "fee_estimates.dat"))
        if self.datadir is not None and a.get_bool("persistmempool", True):  # -persistmempool (LoadMempool)
            n = self.state.load_mempool(os.path.join(self.datadir, "mempool.dat"))
            if n:
                log.log_printf(f"Imported mempool transactions from disk: {n} succeeded")
        # the one miner: the mining service (miner/service.py) on every node — GPU ranks, or this
        # host's CPU devices — with -gpufailrate / -dropshare fault injection around its devices
        self.miner = Miner(self.state, self._start_miner_service(a))
        self.metrics_writer = None
        if a.get("metricslog"):
            path = a.get("metricslog")
            if not os.path.isabs(path) and self.datadir:
                path = os.path.join(self.datadir, path)
            self.metrics_writer = metrics.JsonlWriter(path, float(a.get("metricsinterval", "10"))).start()
        self.connman = None
        self._start_p2p()
        self.zmq = None
        zmq_eps = {t: a.get("zmqpub" + t) for t in ("hashblock", "hashtx", "rawblock", "rawtx", "rawmessage")
                   if a.get("zmqpub" + t)}
        if zmq_eps:
            from .net.zmq_pub import ZmqNotifier

            self.zmq = ZmqNotifier(self.state, zmq_eps)
            self.state.register(self.zmq)
        from .utils.notify import Notifier

        self.notifier = Notifier(a.get("blocknotify"), a.get("walletnotify"), a.get("alertnotify"))
        if self.notifier.block:  # -blocknotify: BlockNotifyCallback on every tip change
            from .chain.state import ValidationInterface

            notifier = self.notifier

            class _BlockNotify(ValidationInterface):
                def updated_block_tip(self, tip, fork, initial_download: bool) -> None:
                    notifier.block_tip(tip.hash[::-1].hex(), initial_download)

            self.state.register(_BlockNotify())
        for w in self.wallets.values() if self.notifier.wallet else ():
            if w.history is not None:
                w.history.on_change = lambda txid: self.notifier.wallet_tx(txid[::-1].hex())
        stop_at = a.get_int("stopatheight", 0)
        if stop_at > 0:  # -stopatheight (src/validation.cpp:11280): shut down once the tip reaches it
            from .chain.state import ValidationInterface

            node = self

            class _StopAt(ValidationInterface):
                def updated_block_tip(self, tip, fork, initial_download: bool) -> None:
                    if tip.height >= stop_at:
                        log.log_printf(f"-stopatheight {stop_at} reached")
                        node.request_shutdown()

            self.state.register(_StopAt())
        if a.get_list("loadblock"):
            self._import_blocks(a.get_list("loadblock"))
        self.table.warmup = None
        log.log_printf(f"nodexad started: network={self.network} height={self.state.height()} "
                       f"kawpow_activation={self.params.kawpow_activation_time} gpus={self.gpus or 'none'}")
        if a.get_bool("gen", False) and self.network != "regtest":
            self.miner.set_generate(True, self.mining_script)

    def _start_miner_service(self, a: ArgsManager):
        """The mining service (miner/service.py): one rank per GPU of `-gpus`, this node being rank 0.
        Ranks 1..n-1 are spawned as child processes here, before this process touches a GPU; under
        torchrun (WORLD_SIZE > 1 in the environment) the launcher made them and this is its rank 0.
        Without GPUs the same loop runs on this host's CPU devices: one rank and no process group,
        or `-minerservice -minerranks=N` processes over gloo (rehearsals of the multi-GPU path)."""
        from .miner import service as MS
        from .parallel import world as W

        cpu = not self.gpus
        timeout = float(a.get("minercollectivetimeout", "60"))
        fail, drop = float(a.get("gpufailrate", "0") or 0), float(a.get("dropshare", "0") or 0)
        self.miner_procs = []
        ranks = max(1, a.get_int("minerranks", 1)) if a.get_bool("minerservice", False) else 1
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            W.init(use_gpu=not cpu, timeout_s=max(int(timeout), W.rendezvous_timeout()), elastic=True,
                   collective_timeout_s=timeout)
        elif cpu and ranks == 1 and not a.get_bool("minerforcecollectives", False):
            pass  # a single host rank: nothing to exchange, no process group
        else:
            gpus = self.gpus or [0] * ranks
            if len(gpus) > 1:
                import socket

                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    port = sk.getsockname()[1]
                os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
                env = {"NODEXA_MINER_COLLECTIVE_TIMEOUT": str(timeout),
                       "NODEXA_MINER_WATCHDOG": a.get("minerwatchdog", "120"),
                       "NODEXA_MINER_MAXFAILURES": str(a.get_int("minermaxfailures", 3)),
                       "NODEXA_MINER_FAILRATE": str(fail), "NODEXA_MINER_DROPSHARE": str(drop)}
                if a.get("gpuintensity"):
                    env["NODEXA_MINER_WINDOW"] = a.get("gpuintensity")
                self.miner_procs = MS.spawn_followers(gpus, port, cpu=cpu, extra_env=env)
            W.init(use_gpu=not cpu, timeout_s=max(int(timeout), W.rendezvous_timeout()),
                   device_index=None if cpu else gpus[0],
                   rank=0, world_size=len(gpus), elastic=True, collective_timeout_s=timeout,
                   force_collectives=a.get_bool("minerforcecollectives", False) or None)
        w = W.get()
        window = a.get_int("gpuintensity", 4096 if cpu else 1 << 25)
        dev = MS.make_rank_device(cpu, None if cpu else w.device.index, collective_dag=w.collective, window=window,
                                  fail_rate=fail, drop_rate=drop, seed=0)
        leader = MS.ChainLeader(self.state, target_bits=a.get_int("minertargetbits", 0),
                                state_path=os.path.join(self.datadir, "miner_state.json") if self.datadir else None)
        log.log_printf(f"miner service: {w.world_size} rank(s), backend {w.backend}, "
                       f"{'cpu' if cpu else 'gpu'} devices, {window} nonces per window")
        return MS.MiningService(dev, leader, window=window, watchdog_s=float(a.get("minerwatchdog", "120")),
                                collective_timeout_s=timeout, max_failures=a.get_int("minermaxfailures", 3)).start()

    def params_assume_valid(self) -> str | None:
        """consensus.defaultAssumeValid: none is set for these networks here (the reference's main
        value names a block of its own chain, which a fresh datadir would not have)."""
        return None

    def _apply_vbparams(self, spec: str) -> None:
        if self.network != "regtest":
            raise SystemExit("Version bits parameters may only be overridden on regtest.")
        import dataclasses

        parts = spec.split(":")
        if len(parts) != 3:
            raise SystemExit("Version bits parameters malformed, expecting deployment:start:end")
        name, start, end = parts[0], int(parts[1]), int(parts[2])
        vb = self.state.versionbits
        for i, d in enumerate(vb.deployments):
            if d.name == name:
                vb.deployments = list(vb.deployments)
                vb.deployments[i] = dataclasses.replace(d, start=start, timeout=end)
                vb._cache.clear()
                log.log_printf(f"Setting version bits activation parameters for {name} to start={start}, timeout={end}")
                return
        raise SystemExit(f"Invalid deployment ({name})")

    def _verify_db(self, nblocks: int, level: int) -> None:
        """CVerifyDB at start-up (-checkblocks / -checklevel): the last blocks must read back,
        pass CheckBlock and their proof of work (level >= 1), and have undo data (level >= 2)."""
        st = self.state
        tip = st.tip()
        if nblocks <= 0 or tip is None or tip.height == 0 or st.store is None:
            return
        for h in range(max(1, tip.height - nblocks + 1), tip.height + 1):
            idx = st.chain.at_height(h)
            blk = st.get_block(idx.hash)
            if blk is None:
                raise SystemExit(f"Corrupted block database detected: block {h} unreadable (use -reindex)")
            if level >= 1 and not (_core.check_block(blk, self.params, True)[0]
                                   and _core.check_proof_of_work(st.block_hash(blk.header), blk.header.bits, self.params)):
                raise SystemExit(f"Corrupted block database detected: block {h} invalid (use -reindex)")
            if level >= 2:
                try:
                    ok = st.undo.read(idx.hash, idx.prev_hash) is not None
                except IOError:
                    ok = False
                if not ok:
                    raise SystemExit(f"Corrupted block database detected: bad undo data for block {h} (use -reindex)")
        log.log_printf(f"Verified the last {min(nblocks, tip.height)} blocks at level {level}")

    def _import_blocks(self, files: list[str]) -> None:
        """ThreadImport: -loadblock files, then -stopafterblockimport."""
        st = self.state
        st.importing = True
        try:
            for path in files:
                try:
                    n = st.load_external_block_file(os.path.expanduser(path))
                    log.log_printf(f"Imported {n} blocks from {path}")
                except OSError as e:
                    log.log_printf(f"Warning: Could not open blocks file {path}: {e}")
        finally:
            st.importing = False
        if self.args.get_bool("stopafterblockimport", False):
            log.log_printf("Stopping after block import")
            self.request_shutdown()

    def get_warnings(self) -> str:
        """GetWarnings("rpc") (src/warnings.cpp): -testsafemode, else the unknown-version warning
        the tip update raises when more than half of the last 100 blocks carry version bits no
        known deployment sets (src/validation.cpp UpdateTip)."""
        if self.args.get_bool("testsafemode", False):
            return "testsafemode enabled"
        st = self.state
        if st is None:
            return ""
        tip = st.tip()
        if getattr(self, "_warn_tip", None) != tip.hash:
            self._warn_tip, self._warn = tip.hash, ""
            upgraded, idx = 0, tip
            for _ in range(100):
                if idx is None or idx.height == 0:
                    break
                prev = st.chain.find(idx.prev_hash)
                v = idx.header.version
                if (v & 0xE0000000) == 0x20000000 and (v & ~st.versionbits.block_version(prev)) & 0x1FFFFFFF:
                    upgraded += 1
                idx = prev
            if upgraded > 50:
                self._warn = "Warning: Unknown block versions being mined! It's possible unknown rules are in effect"
        return self._warn

    def observe_safe_mode(self) -> None:
        """ObserveSafeMode (src/rpc/safemode.cpp): a standing warning refuses the RPC, unless
        -disablesafemode."""
        from .rpc.protocol import RPC_FORBIDDEN_BY_SAFE_MODE, RPCError

        w = self.get_warnings()
        if w and not self.args.get_bool("disablesafemode", False):
            raise RPCError(RPC_FORBIDDEN_BY_SAFE_MODE, "Safe mode: " + w)

    def _configure_pruning(self, a) -> None:
        """-prune=<n> (src/init.cpp AppInitParameterInteraction / AppInitMain): 0 keeps every
        block, 1 allows pruneblockchain, a larger n is a target in MiB for automatic pruning."""
        from .chain.state import MIN_DISK_SPACE_FOR_BLOCK_FILES

        st, prune = self.state, a.get_int("prune", 0)
        if prune < 0:
            raise SystemExit("Prune cannot be configured with a negative value.")
        if not prune:
            if st.have_pruned:
                raise SystemExit("You need to rebuild the database using -reindex to go back to unpruned mode.  "
                                 "This will redownload the entire blockchain")
            return
        if a.get_bool("txindex", False):
            raise SystemExit("Prune mode is incompatible with -txindex.")
        if a.get_bool("rescan", False):
            raise SystemExit("Rescans are not possible in pruned mode. You will need to use -reindex which will "
                             "download the whole blockchain again.")
        if st.store is not None and st.db_format != "leveldb":
            raise SystemExit("Prune mode needs the LevelDB block index (-dbformat=leveldb).")
        target = 1 if prune == 1 else prune << 20
        if prune != 1 and target < MIN_DISK_SPACE_FOR_BLOCK_FILES:
            raise SystemExit(f"Prune configured below the minimum of {MIN_DISK_SPACE_FOR_BLOCK_FILES >> 20} MiB.  "
                             "Please use a higher number.")
        st.prune_target = target
        st._check_for_pruning = target > 1  # AppInitMain: look once at start-up
        log.log_printf(f"Prune mode: {'manual (pruneblockchain)' if target == 1 else f'target {prune} MiB'}")

    def _wallet_paths(self, name: str) -> tuple[str | None, str | None]:
        """Files of wallet `name`: the wallet itself (keys, accounts, labels) and its transaction
        history, `<name without .json>_txs.json` (wallet.json -> wallet_txs.json)."""
        if not self.datadir:
            return None, None
        if name.endswith(".dat"):  # -wallet=<name>.dat names a reference wallet: its JSON sits beside it
            name = name[:-4] + ".json"
        stem = name[:-5] if name.endswith(".json") else name
        return os.path.join(self.datadir, name), os.path.join(self.datadir, stem + "_txs.json")

    def _reference_wallet_file(self, name: str, wpath: str | None) -> str | None:
        """The reference wallet.dat (Berkeley DB) to import for wallet `name` (wallet/walletdb.py):
        <datadir>/wallet.dat for the default wallet, <datadir>/<name> for -wallet=<name>.dat; only
        while no JSON wallet of that name exists."""
        from .wallet.walletdb import is_bdb_file

        if not self.datadir or wpath is None or os.path.exists(wpath):
            return None
        dat = "wallet.dat" if name == DEFAULT_WALLET else name if name.endswith(".dat") else None
        if dat is None:
            return None
        path = os.path.join(self.datadir, dat)
        return path if is_bdb_file(path) else None

    def resolve_wallet(self):
        """GetWalletForJSONRPCRequest + EnsureWalletIsAvailable (src/wallet/rpcwallet.cpp:40-78): the
        wallet a request's /wallet/<name> endpoint names, the only wallet, or an error."""
        from .rpc.protocol import (REQUEST_WALLET, RPC_METHOD_NOT_FOUND, RPC_WALLET_NOT_FOUND,
                                   RPC_WALLET_NOT_SPECIFIED, RPCError)

        if not self.wallets:
            raise RPCError(RPC_METHOD_NOT_FOUND, "Method not found (wallet disabled)")
        name = REQUEST_WALLET.get()
        if name:
            w = self.wallets.get(name)
            if w is None:
                raise RPCError(RPC_WALLET_NOT_FOUND, "Requested wallet does not exist or is not loaded")
            return w
        if name == "" and len(self.wallets) > 1:
            raise RPCError(RPC_WALLET_NOT_SPECIFIED,
                           "Wallet file not specified (must request wallet RPC through /wallet/<filename> uri-path).")
        return next(iter(self.wallets.values()))  # the only wallet, or the default outside a request

    @property
    def wallet(self):
        """The wallet of the current request (see resolve_wallet), None where there is none to
        name: no wallet loaded, or several and the request did not pick one."""
        from .rpc.protocol import RPCError

        try:
            return self.resolve_wallet()
        except RPCError as e:
            if e.code == -18:
                raise
            return None

    @property
    def asset_wallet(self):
        return self._asset_wallets.get(getattr(self.wallet, "name", None))

    def asset_wallet_instance(self):
        """The request wallet's AssetWallet, built on first use (shared by the asset, message and
        reward RPCs)."""
        w = self.resolve_wallet()
        aw = self._asset_wallets.get(w.name)
        if aw is None:
            from .wallet.assets import AssetWallet

            aw = self._asset_wallets[w.name] = AssetWallet(w)
        return aw

    def _start_p2p(self) -> None:
        """-listen / -port / -bind / -connect (CConnman subset, net/p2p.py). Listening is opt-in
        (-listen or -port) so tests and benches never fight over the default port."""
        from .chain.state import ValidationInterface
        from .net.p2p import ConnectionManager

        a = self.args
        from .net.netbase import parse_host_port

        listen = None
        port = a.get_int("port", self.params.default_port)
        binds = [parse_host_port(b, port) + (False,) for b in a.get_list("bind")]
        binds += [parse_host_port(b, port) + (True,) for b in a.get_list("whitebind")]  # -whitebind=addr:port
        if a.get_bool("listen", False) or a.is_set("port") or binds:
            first = binds.pop(0) if binds and not binds[0][2] else None
            listen = (first[0], first[1]) if first else (("127.0.0.1", port) if not binds else None)
        connect = a.get_list("connect")
        seeds, adds = a.get_list("seednode"), a.get_list("addnode")
        if listen is None and not binds and not connect and not seeds and not adds:
            return
        self.connman = ConnectionManager(self.state, self.params, gpus=self.gpus, listen=listen,
                                         verify_mode=a.get("p2pverifymode", "auto"), datadir=self.datadir,
                                         connect_only=bool(connect),
                                         max_outbound=a.get_int("maxconnections", 8) if not connect else 0)
        self.connman.proxies.configure(a)
        self.connman.extra_binds = binds
        self.connman.max_receive_buffer = a.get_int("maxreceivebuffer", 5000) * 1000
        self.connman.max_send_buffer = a.get_int("maxsendbuffer", 1000) * 1000
        self.connman.drop_messages_test = max(0, a.get_int("dropmessagestest", 0))
        self.connman.allow_dns = a.get_bool("dns", True)
        import collections

        self.connman.extra_txn = collections.deque(maxlen=max(0, a.get_int("blockreconstructionextratxn", 100)))
        from .net import protocol as P
        from .rpc.server import parse_allow_subnets

        self.connman.whitelist = parse_allow_subnets(a.get_list("whitelist"))
        self.connman.blocks_only = a.get_bool("blocksonly", False)
        self.connman.max_orphans = a.get_int("maxorphantx", self.connman.max_orphans)
        self.connman.max_outbound_limit = a.get_int("maxuploadtarget", 0) * 1024 * 1024  # MiB per 24 h
        from .net.timedata import DEFAULT_MAX_TIME_ADJUSTMENT, TimeData

        self.connman.timedata = TimeData(max(0, a.get_int("maxtimeadjustment", DEFAULT_MAX_TIME_ADJUSTMENT)))
        if a.get_bool("dnsseed", not connect) and not a.get_list("connect"):  # -dnsseed (off with -connect)
            self.connman.dns_seeds = list(DNS_SEEDS.get(self.network, []))
        self.connman.force_dns_seed = a.get_bool("forcednsseed", False)
        self.connman.peer_bloom_filters = a.get_bool("peerbloomfilters", True)
        self.connman.whitelist_relay = a.get_bool("whitelistrelay", True)
        self.connman.whitelist_force_relay = a.get_bool("whitelistforcerelay", True)
        self.connman.user_agent = P.user_agent(a.get_list("uacomment"))
        self.connman.start()
        cm = self.connman
        if listen is not None and a.get_bool("discover", not a.get_list("externalip") and not a.is_set("bind")):
            cm.discover_local_addresses()  # -discover: Discover() adds this host's routable addresses
        for ext in a.get_list("externalip"):  # -externalip: AddLocal(LOCAL_MANUAL)
            from .net.netbase import parse_host_port

            h, pt = parse_host_port(ext, cm.port or self.params.default_port)
            cm.add_local(h, pt, 4)
        if listen is not None and a.get_bool("upnp", False):  # MapPort(-upnp): net/upnp.py
            from .net.upnp import PortMapper

            self.upnp = PortMapper(cm.port, add_local=cm.add_local,
                                   discover_external=a.get_bool("discover", True))
            self.upnp.start()
        if listen is not None and a.get_bool("listenonion", True):  # StartTorControl (src/init.cpp)
            from .net.torcontrol import DEFAULT_TOR_CONTROL, TorController

            self.torcontrol = TorController(a.get("torcontrol", DEFAULT_TOR_CONTROL), self.datadir, cm.port,
                                            proxies=cm.proxies, add_local=lambda h, p: cm.add_local(h, p, 4),
                                            remove_local=cm.remove_local, password=a.get("torpassword", ""),
                                            onion_arg_set=a.get("onion") is not None)
            self.torcontrol.start()
        st = self.state

        class _Relay(ValidationInterface):
            def transaction_added_to_mempool(self, tx) -> None:
                cm.announce_tx(tx.txid())

            def updated_block_tip(self, tip, fork, initial_download: bool) -> None:
                cm.announce_block(tip.header, st.get_block(tip.hash))

        self.state.register(_Relay())
        # -seednode / -addnode: known to the address manager (ThreadOpenConnections dials them)
        for c in seeds + adds:
            host, _, port = c.rpartition(":")
            cm.addrman.add([(host or "127.0.0.1", int(port), 1, int(time.time()))], "127.0.0.1")
            if c in adds:
                cm.added_nodes.append(c)
        for c in connect:
            host, _, port = c.rpartition(":")
            try:
                cm.connect(host or "127.0.0.1", int(port))
            except OSError as e:
                log.log_printf(f"connect to {c} failed: {e}")

    def _start_rpc(self) -> None:
        a = self.args
        creds = []
        user, pw = a.get("rpcuser"), a.get("rpcpassword")
        if user and pw:
            creds.append(f"{user}:{pw}")
        elif self.datadir is not None and not a.get_list("rpcauth"):
            creds.append(make_cookie(self.datadir, a.get("rpccookiefile")))
        port = a.get_int("rpcport", self.params.default_rpc_port)
        host = a.get("rpcbind", "127.0.0.1")
        from .rpc.server import parse_allow_subnets

        self.rpc = RPCServer(self.table, host, port, creds, a.get_int("rpcworkqueue", 16),
                             rest=self.rest if a.get_bool("rest", False) else None,  # -rest (DEFAULT_REST_ENABLE=false)
                             rpcauth=a.get_list("rpcauth"), allow=parse_allow_subnets(a.get_list("rpcallowip")),
                             threads=a.get_int("rpcthreads", 4), idle_timeout=float(a.get("rpcservertimeout", "30")),
                             # -webgui: the wallet page at http://<rpcbind>:<rpcport>/gui (off by default:
                             # a browser that saved the RPC credentials is a CSRF target, rpc/server.py)
                             gui=os.path.join(os.path.dirname(os.path.abspath(__file__)), "gui", "index.html")
                             if a.get_bool("webgui", False) else None)
        self.rpc.start()
        log.log_printf(f"RPC listening on {host}:{self.rpc.port}")

    def request_shutdown(self) -> None:
        self._shutdown.set()

    def shutdown_requested(self) -> bool:
        return self._shutdown.is_set()

    def wait(self) -> None:
        while not self._shutdown.wait(0.5):
            pass

    def stop(self) -> None:
        if getattr(self, "_stopped", False):
            return
        self._stopped = True
        if self.miner is not None:
            self.miner.close()
            if self.miner.service is not None:
                for p in getattr(self, "miner_procs", []):
                    try:
                        p.wait(timeout=30)
                    except Exception:  # noqa: BLE001 — a follower that does not stop is killed
                        p.kill()
                from .parallel import world as W

                W.shutdown()
        if self.state is not None and self.datadir is not None and self.args.get_bool("persistmempool", True):
            try:
                self.state.save_mempool(os.path.join(self.datadir, "mempool.dat"))  # DumpMempool on shutdown
            except OSError as e:
                log.log_printf(f"Failed to dump mempool: {e}")
        if self.state is not None and self.datadir is not None:
            try:  # Shutdown: FlushUnconfirmed, then fee_estimates.dat
                self.state.save_fee_estimates(os.path.join(self.datadir, "fee_estimates.dat"))
            except OSError as e:
                log.log_printf(f"Failed to write fee estimates: {e}")
        if getattr(self, "torcontrol", None) is not None:
            self.torcontrol.stop()  # InterruptTorControl / StopTorControl
        if getattr(self, "upnp", None) is not None:
            self.upnp.stop()  # MapPort(false): the mapping is deleted
        if getattr(self, "connman", None) is not None:
            self.connman.stop()
        if self.state is not None:
            self.state.close()
        if getattr(self, "zmq", None) is not None:
            self.zmq.stop()
        if getattr(self, "metrics_writer", None) is not None:
            self.metrics_writer.stop()
        if self.rpc is not None:
            self.rpc.stop()
        if self.datadir is not None:
            delete_cookie(self.datadir, self.args.get("rpccookiefile"))
        if getattr(self, "_pidfile", None):
            try:
                os.unlink(self._pidfile)  # RemovePidFile
            except OSError:
                pass
            self._pidfile = None
        if self._lock_file is not None:
            fcntl.flock(self._lock_file, fcntl.LOCK_UN)
            self._lock_file.close()
            self._lock_file = None
        log.log_printf("Shutdown: done")

    # ------------------------------------------------------------------ helpers used by RPCs
    def peer_count(self) -> int:
        return self.connman.peer_count() if getattr(self, "connman", None) is not None else 0

    def blocks_size_on_disk(self) -> int:
        if self.datadir is None:
            return 0
        bdir = os.path.join(self.datadir, "blocks")
        return sum(os.path.getsize(os.path.join(bdir, f)) for f in os.listdir(bdir)) if os.path.isdir(bdir) else 0

    def template_for_gbt(self):
        script = self.mining_script or bytes([0x51])  # OP_TRUE when no -miningaddress (src/rpc/mining.cpp:550-563)
        tpl = BlockAssembler(self.state).create_new_block(script)
        ExtraNonce().increment(tpl.block, tpl.height)
        return tpl

    def register_equihash_template(self, tpl) -> dict:
        """The Equihash extension's template cache (the analogue of mapHVNKAWBlockTemplates): keyed by
        the 80-byte input prefix, which an external solver extends with its nonce256."""
        hdr = tpl.block.header
        prefix = hdr.kawpow_input()
        key = prefix.hex()
        self.equihash_templates[key] = tpl
        while len(self.equihash_templates) > 64:
            self.equihash_templates.pop(next(iter(self.equihash_templates)))
        return {"n": self.params.equihash_n, "k": self.params.equihash_k, "personalization": "ZcashPoW",
                "input": key, "nonce_bytes": 32, "solution_bytes": _core.EquihashParams(
                    self.params.equihash_n, self.params.equihash_k).solution_bytes,
                "header_version": hdr.version}

    def register_pprpc_template(self, tpl) -> str:
        """mapHVNKAWBlockTemplates: reuse the last header for 30 s (src/rpc/mining.cpp:722-739)."""
        if self._last_pprpc is not None:
            hh, t0 = self._last_pprpc
            old = self.pprpc_templates.get(hh)
            if old is not None and old.block.header.prev == tpl.block.header.prev and tpl.block.header.time - 30 < old.block.header.time:
                return hh
        hh = _core.u256_hex(tpl.block.header.kawpow_header_hash())
        self.pprpc_templates[hh] = tpl
        self._last_pprpc = (hh, time.time())
        if len(self.pprpc_templates) > 64:
            for k in list(self.pprpc_templates)[:-64]:
                self.pprpc_templates.pop(k, None)
        return hh

    def gpu_info(self) -> list[dict]:
        """getmininginfo.gpus[]: every rank of the miner world (rate, shares, stale rate, resident
        epochs, device / step / collective times, failures), plus this GPU's properties."""
        svc = self.miner.service if self.miner else None
        if svc is None:
            return []
        out = svc.rank_info()
        for g in out:
            g["intensity"] = svc.window
            g["ranks"] = svc.world_size
        if out and self.gpus:
            try:
                from .ops import runtime

                out[0].update(runtime.hip().device_props(self.gpus[0]))
            except Exception as e:  # pragma: no cover
                out[0]["error"] = str(e)
        return out

    def gpu_memory_info(self) -> list[dict]:
        out = []
        if not self.gpus:
            return out
        import torch

        for d in self.gpus:
            free, total = torch.cuda.mem_get_info(d)
            out.append({"device": d, "free": free, "total": total})
        return out

    def verify_headers(self, headers) -> list[dict]:
        """Full PoW verification of a header batch (models/verify.py picks GPU or CPU)."""
        from .models import verify

        return list(verify.verify_headers(self.params, headers, gpus=self.gpus))

    def equihash_solve(self, inp: bytes) -> list[list[int]]:
        if self.gpus:
            from .ops.equihash import EquihashSolver

            import torch

            with torch.cuda.device(self.gpus[0]):
                s = EquihashSolver(num_inst=1, device=self.gpus[0])
                return s.solve([inp])[0]
        from .models.equihash import solve_cpu

        return solve_cpu(inp)

    def _rest_getutxos(self, parts: list[str], json):
        """rest_getutxos (src/rest.cpp): which of up to 15 outpoints are unspent, optionally in the
        mempool view. bin = int32 height, tip hash, bitmap, [u32 0, u32 height, CTxOut] per coin."""
        import struct

        def _cs(n: int) -> bytes:  # CompactSize
            if n < 253:
                return bytes([n])
            return b"\xfd" + struct.pack("<H", n) if n <= 0xFFFF else b"\xfe" + struct.pack("<I", n)

        if not parts:
            return 400, "text/plain", b"Error: empty request"
        last, _, fmt = parts[-1].partition(".")
        parts = parts[:-1] + [last]
        check_mempool = parts[0] == "checkmempool"
        if check_mempool:
            parts = parts[1:]
        if fmt not in ("bin", "hex", "json"):
            return 404, "text/plain", b"output format not found (available: .bin, .hex, .json)"
        if not parts or len(parts) > 15:
            return 400, "text/plain", b"Error: max outpoints exceeded (max: 15, tried: %d)" % len(parts)
        st = self.state
        outs = []
        try:
            for q in parts:
                txid, _, n = q.partition("-")
                outs.append((_core.u256_from_hex(txid), int(n)))
        except ValueError:
            return 400, "text/plain", b"Parse error"
        with st.lock:
            tip = st.coins_tip()
            pool_spent = {(i.prevout.hash, i.prevout.n) for e in st.mempool.values() for i in e.tx.vin} \
                if check_mempool else set()
            found = []
            for h, n in outs:
                c = st.coins.get(h, n)
                if c is None and check_mempool and h in st.mempool and n < len(st.mempool[h].tx.vout):
                    o = st.mempool[h].tx.vout[n]
                    c = (o.value, o.script_pubkey, 0x7FFFFFFF, False)  # MEMPOOL_HEIGHT
                if c is not None and (h, n) in pool_spent:
                    c = None
                found.append(c)
        bits = "".join("1" if c is not None else "0" for c in found)
        coins = [c for c in found if c is not None]
        if fmt == "json":
            body = {"chainHeight": tip.height, "chaintipHash": _core.u256_hex(tip.hash), "bitmap": bits,
                    "utxos": [{"height": c[2], "value": c[0] / 1e8,
                               "scriptPubKey": {"hex": c[1].hex()}} for c in coins]}
            return 200, "application/json", json.dumps(body).encode()
        bitmap = bytearray((len(found) + 7) // 8)
        for i, c in enumerate(found):
            if c is not None:
                bitmap[i // 8] |= 1 << (i % 8)
        raw = struct.pack("<i", tip.height) + bytes(tip.hash) + _cs(len(bitmap)) + bytes(bitmap)
        raw += _cs(len(coins))
        for value, spk, height, _ in coins:
            raw += struct.pack("<IIq", 0, height, value) + _cs(len(spk)) + spk
        return (200, "application/octet-stream", raw) if fmt == "bin" else (200, "text/plain", raw.hex().encode())

    def rest(self, path: str):
        """REST (src/rest.cpp:569-580): /rest/chaininfo.json, /rest/block/<hash>.{bin,hex,json},
        /rest/block/notxdetails/<hash>.{bin,hex,json}, /rest/headers/<n>/<hash>.{bin,hex,json},
        /rest/tx/<txid>.{bin,hex,json} (mempool, -txindex or an unspent output), /rest/mempool/{info,contents}.json,
        /rest/blockhashbyheight/<h>.{json,hex,bin}, /rest/getutxos[/checkmempool]/<txid>-<n>/....{bin,hex,json}
        (rest_getutxos: at most 15 outpoints), /rest/metrics (Prometheus)."""
        import json

        parts = path.split("?")[0].split("/")[2:]
        if parts == ["metrics"]:  # Prometheus text exposition of utils/metrics.REGISTRY
            return 200, "text/plain; version=0.0.4", metrics.REGISTRY.prometheus().encode()
        if parts in (["mempool", "info.json"], ["mempool", "contents.json"]):  # src/rest.cpp rest_mempool_*
            mp = self.state.mempool
            if parts[1] == "info.json":
                body = {"size": len(mp), "bytes": sum(len(e.tx.serialize(True)) for e in mp.values())}
            else:
                body = {_core.u256_hex(k): {"fee": e.fee / 1e8, "time": int(e.time)} for k, e in mp.items()}
            return 200, "application/json", json.dumps(body).encode()
        if len(parts) == 2 and parts[0] == "blockhashbyheight":
            h, _, fmt = parts[1].partition(".")
            idx = self.state.chain.at_height(int(h))
            if idx is None:
                return 404, "text/plain", b"Block height out of range"
            if fmt == "json":
                return 200, "application/json", json.dumps({"blockhash": _core.u256_hex(idx.hash)}).encode()
            return (200, "application/octet-stream", bytes(idx.hash)) if fmt == "bin" else \
                (200, "text/plain", _core.u256_hex(idx.hash).encode())
        if parts == ["chaininfo.json"]:
            tip = self.state.tip()
            body = json.dumps({"chain": self.network, "blocks": tip.height, "bestblockhash": _core.u256_hex(tip.hash)})
            return 200, "application/json", body.encode()
        rpc = lambda name, *a: self.table.commands[name].handler(list(a))  # noqa: E731 — JSON forms reuse the RPCs
        if parts[:1] == ["block"] and len(parts) in (2, 3) and (len(parts) == 2 or parts[1] == "notxdetails"):
            h, _, fmt = parts[-1].partition(".")
            raw = self.state.get_block_raw(_core.u256_from_hex(h))
            if raw is None:
                return 404, "text/plain", f"{h} not found".encode()
            if fmt == "json":  # rest_block_extended / rest_block_notxdetails
                return 200, "application/json", json.dumps(rpc("getblock", h, 1 if len(parts) == 3 else 2)).encode()
            return (200, "application/octet-stream", raw) if fmt == "bin" else (200, "text/plain", raw.hex().encode())
        if len(parts) == 3 and parts[0] == "headers":
            n = int(parts[1])
            if n < 1 or n > 2000:
                return 400, "text/plain", f"Header count out of range: {n}".encode()
            h, _, fmt = parts[2].partition(".")
            idx = self.state.chain.find(_core.u256_from_hex(h))
            out, found = b"", []
            while idx is not None and n > 0 and self.state.chain.in_active_chain(idx):
                out += idx.header.serialize(self.params.kawpow_activation_time)
                found.append(idx)
                idx = self.state.chain.at_height(idx.height + 1)
                n -= 1
            if fmt == "json":
                return 200, "application/json", json.dumps([rpc("getblockheader", _core.u256_hex(i.hash)) for i in found]).encode()
            return (200, "application/octet-stream", out) if fmt == "bin" else (200, "text/plain", out.hex().encode())
        if parts and parts[0] == "getutxos":
            return self._rest_getutxos(parts[1:], json)
        if len(parts) == 2 and parts[0] == "tx":  # rest_tx: GetTransaction (pool, -txindex, unspent output)
            h, _, fmt = parts[1].partition(".")
            try:
                raw = bytes.fromhex(rpc("getrawtransaction", h))
            except Exception:  # noqa: BLE001 — not found in any of the places GetTransaction looks
                return 404, "text/plain", f"{h} not found".encode()
            if fmt == "json":
                return 200, "application/json", json.dumps(rpc("getrawtransaction", h, True)).encode()
            return (200, "application/octet-stream", raw) if fmt == "bin" else (200, "text/plain", raw.hex().encode())
        return 404, "text/plain", b"unknown REST path"


def main(argv: list[str] | None = None) -> int:
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and int(os.environ.get("RANK", "0")) != 0:
        # torchrun launched the node on every GPU: ranks >= 1 are mining followers of rank 0
        from .miner.service import follower_main

        return follower_main()
    args = ArgsManager()
    rest = args.parse_parameters(sys.argv[1:] if argv is None else argv)
    if rest:
        print(f"Error: unexpected arguments {rest}", file=sys.stderr)
        return 1
    conf = args.get("conf", "nodexa.conf")
    if args.get("datadir"):
        args.read_config_file(os.path.join(os.path.expanduser(args.get("datadir")), conf))
    node = Node(args)
    signal.signal(signal.SIGTERM, lambda *_: node.request_shutdown())
    signal.signal(signal.SIGINT, lambda *_: node.request_shutdown())
    node.start()
    try:
        node.wait()
    finally:
        node.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())

// HIP host runtime for the gfx950 kernels (pybind11 module `_hip`).
//
// * Code objects (static .hsaco from _build.py, or per-period KawPow objects
//   from ops/jit.py) are loaded with hipModuleLoadData and launched with
//   hipModuleLaunchKernel; each kernel takes one parameter struct from
//   hip/kernels/kernel_params.h, so host and device share the ABI header.
// * Device memory and streams belong to torch (its caching allocator, its
//   streams, its RCCL communicators): every entry point takes raw device
//   pointers and a hipStream_t as integers. This module links the very same
//   libamdhip64.so torch loaded, so those handles are valid here.
// * Launches never synchronise and never allocate, so callers may capture
//   them into hipGraphs.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>

#include "../kernels/kernel_params.h"

namespace py = pybind11;

namespace {

void check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}


FastMod32 make_fastmod(uint32_t d) {
    if (d < 2) throw std::invalid_argument("fastmod divisor must be >= 2");
    uint32_t s = 0;
    while ((uint64_t(1) << s) < d) ++s;  // s = ceil(log2 d)
    const uint64_t m = ((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1;
    FastMod32 f{};
    f.d = d;
    f.m = uint32_t(m);
    f.s = s;
    f.mb = uint32_t((uint64_t(1) << 32) / d);
    f.m24 = (d > (1u << 16) && d < (1u << 24)) ? uint32_t((uint64_t(1) << 40) / d) : 0u;
    return f;
}

struct Kernel {
    hipFunction_t fn = nullptr;
    std::string name;
    int device = -1;
    int max_threads = 0;  // __launch_bounds__ of the kernel = the block size its launcher uses

    void launch_bytes(dim3 grid, dim3 block, unsigned shmem, hipStream_t stream, const void* params,
                      size_t size) const {
        int cur = -1;
        check(hipGetDevice(&cur), "hipGetDevice");
        if (cur != device)
            throw std::runtime_error("kernel " + name + " belongs to device " + std::to_string(device) +
                                     " but current device is " + std::to_string(cur));
        void* config[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, const_cast<void*>(params), HIP_LAUNCH_PARAM_BUFFER_SIZE,
                          &size, HIP_LAUNCH_PARAM_END};
        check(hipModuleLaunchKernel(fn, grid.x, grid.y, grid.z, block.x, block.y, block.z, shmem, stream, nullptr,
                                    config),
              ("hipModuleLaunchKernel(" + name + ")").c_str());
    }
    // kernelParams form (argv[i] = pointer to argument i). Used under stream capture with argv and
    // the argument storage owned by the graph, so no node can refer to a dead stack frame.
    void launch_args(dim3 grid, dim3 block, unsigned shmem, hipStream_t stream, void** argv) const {
        check(hipModuleLaunchKernel(fn, grid.x, grid.y, grid.z, block.x, block.y, block.z, shmem, stream, argv,
                                    nullptr),
              ("hipModuleLaunchKernel(" + name + ")").c_str());
    }
};

struct CodeObject {
    hipModule_t mod = nullptr;
    int device = -1;
    std::string image;  // kept alive for the module's lifetime
    std::mutex mu;
    std::unordered_map<std::string, std::shared_ptr<Kernel>> fns;

    explicit CodeObject(std::string img) : image(std::move(img)) {
        check(hipGetDevice(&device), "hipGetDevice");
        check(hipModuleLoadData(&mod, image.data()), "hipModuleLoadData");
    }
    ~CodeObject() {
        if (mod) (void)hipModuleUnload(mod);
    }
    std::shared_ptr<Kernel> function(const std::string& name) {
        std::lock_guard<std::mutex> g(mu);
        auto it = fns.find(name);
        if (it != fns.end()) return it->second;
        auto k = std::make_shared<Kernel>();
        check(hipModuleGetFunction(&k->fn, mod, name.c_str()), ("hipModuleGetFunction(" + name + ")").c_str());
        k->name = name;
        k->device = device;
        check(hipFuncGetAttribute(&k->max_threads, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, k->fn),
              "hipFuncGetAttribute(MAX_THREADS_PER_BLOCK)");
        fns[name] = k;
        return k;
    }
};

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// Two 32-byte hashes as 8 LE words.
void load_words(const std::string& b, uint32_t out[8]) {
    if (b.size() != 32) throw std::invalid_argument("expected 32-byte header hash");
    std::memcpy(out, b.data(), 32);
}

}  // namespace


PYBIND11_MODULE(_hip, m) {
    m.doc() = "nodexa HIP host runtime: gfx950 code-object loading and typed kernel launchers";

    m.def("device_count", [] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) return 0;
        return n;
    });
    m.def("set_device", [](int d) { check(hipSetDevice(d), "hipSetDevice"); });
    m.def("get_device", [] {
        int d = -1;
        check(hipGetDevice(&d), "hipGetDevice");
        return d;
    });
    m.def("synchronize", [] { check(hipDeviceSynchronize(), "hipDeviceSynchronize"); },
          py::call_guard<py::gil_scoped_release>());
    m.def("stream_synchronize", [](uintptr_t s) { check(hipStreamSynchronize(as_stream(s)), "hipStreamSynchronize"); },
          py::call_guard<py::gil_scoped_release>());
    m.def("device_name", [](int d) {
        hipDeviceProp_t p;
        check(hipGetDeviceProperties(&p, d), "hipGetDeviceProperties");
        return std::string(p.gcnArchName);
    });
    m.def("device_props", [](int d) {
        hipDeviceProp_t p;
        check(hipGetDeviceProperties(&p, d), "hipGetDeviceProperties");
        py::dict r;
        r["name"] = std::string(p.name);
        r["arch"] = std::string(p.gcnArchName);
        r["cus"] = p.multiProcessorCount;
        r["total_mem"] = p.totalGlobalMem;
        r["l2_bytes"] = p.l2CacheSize;
        r["lds_per_block"] = p.sharedMemPerBlock;
        r["clock_khz"] = p.clockRate;
        r["mem_clock_khz"] = p.memoryClockRate;
        r["mem_bus_width"] = p.memoryBusWidth;
        return r;
    });
    // Thin stream-ordered helpers for pipelines issued from Python (ops/header_batch.py): one
    // pybind call each instead of torch's Python-level stream / event / copy wrappers.
    m.def("event_create", [](bool timing) {
        hipEvent_t e;
        check(hipEventCreateWithFlags(&e, timing ? hipEventDefault : hipEventDisableTiming), "hipEventCreate");
        return reinterpret_cast<uintptr_t>(e);
    }, py::arg("timing") = false);
    m.def("event_destroy", [](uintptr_t e) { check(hipEventDestroy(reinterpret_cast<hipEvent_t>(e)), "hipEventDestroy"); });
    m.def("event_record", [](uintptr_t e, uintptr_t s) {
        check(hipEventRecord(reinterpret_cast<hipEvent_t>(e), as_stream(s)), "hipEventRecord");
    });
    m.def("stream_wait_event", [](uintptr_t s, uintptr_t e) {
        check(hipStreamWaitEvent(as_stream(s), reinterpret_cast<hipEvent_t>(e), 0), "hipStreamWaitEvent");
    });
    m.def("event_synchronize", [](uintptr_t e) {
        check(hipEventSynchronize(reinterpret_cast<hipEvent_t>(e)), "hipEventSynchronize");
    }, py::call_guard<py::gil_scoped_release>());
    m.def("event_elapsed_ms", [](uintptr_t a, uintptr_t b) {
        float ms = 0;
        check(hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(a), reinterpret_cast<hipEvent_t>(b)), "hipEventElapsedTime");
        return ms;
    });
    // kind: "htod" / "dtoh" / "dtod" (an explicit direction spares the runtime a pointer lookup)
    m.def("memcpy_async", [](uintptr_t dst, uintptr_t src, size_t n, uintptr_t s, const std::string& kind) {
        const hipMemcpyKind k = kind == "htod" ? hipMemcpyHostToDevice
                                : kind == "dtoh" ? hipMemcpyDeviceToHost
                                : kind == "dtod" ? hipMemcpyDeviceToDevice
                                                 : throw std::invalid_argument("memcpy_async kind: htod, dtoh or dtod");
        if (n) check(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n, k, as_stream(s)),
                     "hipMemcpyAsync");
    }, py::arg("dst"), py::arg("src"), py::arg("n"), py::arg("stream"), py::arg("kind"));
    m.def("memset_async", [](uintptr_t dst, int v, size_t n, uintptr_t s) {
        if (n) check(hipMemsetAsync(reinterpret_cast<void*>(dst), v, n, as_stream(s)), "hipMemsetAsync");
    });
    m.def("memcpy_htod", [](uintptr_t dst, uintptr_t src, size_t n) {
        check(hipMemcpy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n, hipMemcpyHostToDevice),
              "hipMemcpy(HtoD)");
    }, py::call_guard<py::gil_scoped_release>());
    m.def("memcpy_dtoh", [](uintptr_t dst, uintptr_t src, size_t n) {
        check(hipMemcpy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n, hipMemcpyDeviceToHost),
              "hipMemcpy(DtoH)");
    }, py::call_guard<py::gil_scoped_release>());
    m.def("fastmod32", [](uint32_t d) {
        FastMod32 f = make_fastmod(d);
        return py::make_tuple(f.d, f.m, f.s);
    });
    m.def("fastmod32_eval", [](uint32_t x, uint32_t d) {
        FastMod32 f = make_fastmod(d);
        const uint32_t t = uint32_t((uint64_t(x) * f.m) >> 32);
        const uint32_t q = (t + ((x - t) >> 1)) >> (f.s - 1);
        return x - q * f.d;
    }, "host model of the device FastMod32 (tests compare it with x % d)");
    m.def("sizeof_results", [] { return sizeof(KawpowResults); });
    m.def("sizeof_share", [] { return sizeof(KawpowShare); });
    m.attr("KAWPOW_MAX_SHARES") = NODEXA_KAWPOW_MAX_SHARES;
    m.attr("KAWPOW_BLOCK") = NODEXA_KAWPOW_BLOCK;

    py::class_<Kernel, std::shared_ptr<Kernel>>(m, "Kernel")
        .def_readonly("name", &Kernel::name)
        .def_readonly("device", &Kernel::device)
        .def_readonly("max_threads", &Kernel::max_threads)
        .def("launch", [](const Kernel& k, std::tuple<unsigned, unsigned, unsigned> g,
                          std::tuple<unsigned, unsigned, unsigned> b, unsigned shmem, uintptr_t stream,
                          const py::bytes& params) {
            std::string p = params;
            k.launch_bytes(dim3(std::get<0>(g), std::get<1>(g), std::get<2>(g)),
                           dim3(std::get<0>(b), std::get<1>(b), std::get<2>(b)), shmem, as_stream(stream),
                           p.data(), p.size());
        }, "generic launch with a packed parameter struct");

    py::class_<CodeObject, std::shared_ptr<CodeObject>>(m, "CodeObject")
        .def(py::init([](const py::bytes& img) { return std::make_shared<CodeObject>(std::string(img)); }))
        .def_readonly("device", &CodeObject::device)
        .def("function", &CodeObject::function);

    // ---- typed launchers (layout from kernel_params.h) ----
    m.def("launch_ethash_dag_build", [](const Kernel& k, uintptr_t light, uint32_t light_items, uintptr_t dag,
                                        uint64_t first_item, uint64_t num_items, uintptr_t stream) {
        struct {
            EthashDagParams p;
            FastMod32 lmod;
        } args{};
        args.p.light = reinterpret_cast<const void*>(light);
        args.p.dag = reinterpret_cast<void*>(dag);
        args.p.first_item = first_item;
        args.p.num_items = num_items;
        args.p.light_items = light_items;
        args.lmod = make_fastmod(light_items);
        const unsigned block = 256;  // one item per lane quad (hip/kernels/ethash_dag.hip): 64 per workgroup
        const uint64_t grid = (num_items + 63) / 64;
        if (grid == 0) return;
        if (grid > 0x7fffffffULL) throw std::invalid_argument("dag build launch too large; split it");
        k.launch_bytes(dim3(unsigned(grid)), dim3(block), 0, as_stream(stream), &args, sizeof(args));
    });

    m.def("launch_kawpow_search", [](const Kernel& k, uintptr_t dag, uint32_t dag_items2048, uintptr_t results,
                                     const py::bytes& header, uint64_t start_nonce, uint64_t target,
                                     uint64_t num_nonces, uintptr_t stream, uintptr_t scratch,
                                     uint64_t scratch_bytes, uintptr_t gen_word, uint32_t generation) {
        // search variants are compiled for different block sizes (KP_BLOCK); their
        // __launch_bounds__ is the block, one nonce per thread
        const unsigned block = unsigned(k.max_threads);
        if (block == 0 || num_nonces % block)
            throw std::invalid_argument("num_nonces must be a multiple of the kernel's block size");
        // variants that park digests in HBM write 32 B per nonce of the launch
        if (scratch == 0 || scratch_bytes < num_nonces * 32)
            throw std::invalid_argument("search scratch must hold 32 bytes per nonce");
        KawpowSearchParams p{};
        p.scratch = reinterpret_cast<uint32_t*>(scratch);
        p.dag = reinterpret_cast<const void*>(dag);
        p.results = reinterpret_cast<KawpowResults*>(results);
        p.start_nonce = start_nonce;
        p.target = target;
        load_words(header, p.header);
        p.items = make_fastmod(dag_items2048);
        p.gen_word = reinterpret_cast<const uint32_t*>(gen_word);
        p.generation = generation;
        const uint64_t grid = num_nonces / block;
        if (grid == 0 || grid > 0x7fffffffULL) throw std::invalid_argument("bad search grid");
        k.launch_bytes(dim3(unsigned(grid)), dim3(block), 0, as_stream(stream), &p, sizeof(p));
    }, py::arg("kernel"), py::arg("dag"), py::arg("dag_items2048"), py::arg("results"), py::arg("header"),
       py::arg("start_nonce"), py::arg("target"), py::arg("num_nonces"), py::arg("stream"), py::arg("scratch"),
       py::arg("scratch_bytes"), py::arg("gen_word") = 0, py::arg("generation") = 0);

    // Host-mapped words (fine-grained, coherent pinned memory): the miner's stale-work generation
    // word that running search kernels poll once per workgroup. The pointer is valid on the host
    // and, under HIP's unified addressing, in device code of every GPU of the process.
    m.def("host_words_alloc", [](size_t n) {
        void* p = nullptr;
        check(hipHostMalloc(&p, n * 4, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable),
              "hipHostMalloc(words)");
        std::memset(p, 0, n * 4);
        void* d = nullptr;
        check(hipHostGetDevicePointer(&d, p, 0), "hipHostGetDevicePointer");
        if (d != p) {
            (void)hipHostFree(p);
            throw std::runtime_error("host-mapped word has a different device address (no unified addressing)");
        }
        return reinterpret_cast<uintptr_t>(p);
    });
    m.def("host_words_free", [](uintptr_t p) { check(hipHostFree(reinterpret_cast<void*>(p)), "hipHostFree"); });
    m.def("host_word_store", [](uintptr_t p, size_t i, uint32_t v) {
        __atomic_store_n(reinterpret_cast<uint32_t*>(p) + i, v, __ATOMIC_SEQ_CST);
    });
    m.def("host_word_load", [](uintptr_t p, size_t i) {
        return __atomic_load_n(reinterpret_cast<const uint32_t*>(p) + i, __ATOMIC_SEQ_CST);
    });

    m.def("launch_kawpow_hash_batch", [](const Kernel& k, uintptr_t dag, uint32_t dag_items2048, uintptr_t jobs,
                                         uint32_t num_jobs, uintptr_t out, uintptr_t stream) {
        KawpowHashParams p{};
        p.dag = reinterpret_cast<const void*>(dag);
        p.jobs = reinterpret_cast<const KawpowVerifyJob*>(jobs);
        p.out = reinterpret_cast<uint32_t*>(out);
        p.num_jobs = num_jobs;
        p.items = make_fastmod(dag_items2048);
        const unsigned block = unsigned(k.max_threads);
        const unsigned grid = (num_jobs + block - 1) / block;
        if (grid == 0) return;
        k.launch_bytes(dim3(grid), dim3(block), 0, as_stream(stream), &p, sizeof(p));
    });
    // Classic Ethash hashimoto (ethash_hashimoto.hip): seed -> mix (per_row jobs per 16-lane row,
    // 16 rows per block) -> final, in order on one stream; `seeds` holds n x 64 bytes. Search mode
    // (search_header given, jobs ignored): job i is (header, start_nonce + i); with a boundary, the
    // final kernel appends every job whose final hash is <= it to `hits` ([0] count, then indices).
    m.def("launch_ethash_hash_batch", [](const Kernel& k_seed, const Kernel& k_mix, const Kernel& k_final,
                                         uintptr_t dag, uint32_t full_items, uintptr_t jobs, uint32_t num_jobs,
                                         uintptr_t out, uintptr_t seeds, uintptr_t stream, uint32_t per_row,
                                         const std::string& search_header, uint64_t start_nonce,
                                         const std::string& search_boundary, uintptr_t hits, uint32_t max_hits) {
        // per_row: the mix kernel's hashes per 16-lane row (EH_HASHES, ops/ethash.EH_HASHES)
        if (num_jobs == 0) return;
        if (per_row == 0 || per_row > 16) throw std::invalid_argument("hashes per row in 1..16");
        for (const Kernel* k : {&k_seed, &k_mix, &k_final})
            if (k->max_threads < 256) throw std::invalid_argument("ethash hashimoto kernels need 256-thread blocks");
        EthashHashParams p{};
        p.dag = reinterpret_cast<const void*>(dag);
        p.jobs = reinterpret_cast<const KawpowVerifyJob*>(jobs);
        p.out = reinterpret_cast<uint32_t*>(out);
        p.seeds = reinterpret_cast<uint32_t*>(seeds);
        p.num_jobs = num_jobs;
        p.pages = make_fastmod(full_items);
        if (!search_header.empty() || !search_boundary.empty()) {
            if (search_header.size() != 32 || (!search_boundary.empty() && search_boundary.size() != 32))
                throw std::invalid_argument("search: 32-byte header hash and boundary");
            if (!search_boundary.empty() && (hits == 0 || max_hits == 0))
                throw std::invalid_argument("search: a hit buffer");
            std::memcpy(p.header, search_header.data(), 32);
            if (!search_boundary.empty()) {
                std::memcpy(p.boundary, search_boundary.data(), 32);
                p.hits = reinterpret_cast<uint32_t*>(hits);
                p.max_hits = max_hits;
            }
            p.jobs = nullptr;
            p.start_nonce = start_nonce;
        } else if (jobs == 0) {
            throw std::invalid_argument("jobs, or a search header");
        }
        const hipStream_t s = as_stream(stream);
        const unsigned lanes_grid = (num_jobs + 255) / 256;
        const unsigned per_block = 16 * per_row;
        k_seed.launch_bytes(dim3(lanes_grid), dim3(256), 0, s, &p, sizeof(p));
        k_mix.launch_bytes(dim3((num_jobs + per_block - 1) / per_block), dim3(256), 0, s, &p, sizeof(p));
        k_final.launch_bytes(dim3(lanes_grid), dim3(256), 0, s, &p, sizeof(p));
    }, py::arg("k_seed"), py::arg("k_mix"), py::arg("k_final"), py::arg("dag"), py::arg("full_items"), py::arg("jobs"),
       py::arg("num_jobs"), py::arg("out"), py::arg("seeds"), py::arg("stream"), py::arg("per_row"),
       py::arg("search_header") = std::string(), py::arg("start_nonce") = 0, py::arg("search_boundary") = std::string(),
       py::arg("hits") = 0, py::arg("max_hits") = 0);
    // X16R / X16RV2 (x16r.hip): the 16 chain steps of a batch, each ONE launch with every slot group
    // of the step (x16r_step_all, grid y = slot). order: 16 x n header indices grouped by slot,
    // offsets: 16 x 17 group bounds (device copies; offsets_host is the same table, for the grids).
    m.def("launch_x16r_chain_all", [](const Kernel& k, uintptr_t headers, uintptr_t state, uintptr_t v2,
                                      uintptr_t order, uintptr_t offsets, const std::vector<int32_t>& offsets_host,
                                      uint32_t n, uintptr_t stream) {
        if (n == 0) return;
        if (offsets_host.size() != 16 * 17) throw std::invalid_argument("16 x 17 offsets");
        X16rStepParams p{};
        p.headers = reinterpret_cast<const uint8_t*>(headers);
        p.state = reinterpret_cast<uint8_t*>(state);
        p.v2 = reinterpret_cast<const uint8_t*>(v2);
        p.n = n;
        const hipStream_t st = as_stream(stream);
        const unsigned block = unsigned(k.max_threads);
        for (uint32_t s = 0; s < 16; ++s) {
            int32_t maxg = 0;
            for (int a = 0; a < 16; ++a) {
                const int32_t lo = offsets_host[size_t(s * 17 + a)], hi = offsets_host[size_t(s * 17 + a + 1)];
                if (lo < 0 || hi < lo || uint32_t(hi) > n) throw std::invalid_argument("X16R offsets out of order");
                maxg = std::max(maxg, hi - lo);
            }
            if (maxg == 0) continue;
            p.step = s;
            p.order = reinterpret_cast<const int32_t*>(order) + size_t(s) * n;
            p.offsets = reinterpret_cast<const int32_t*>(offsets) + size_t(s) * 17;
            k.launch_bytes(dim3((uint32_t(maxg) + block - 1) / block, 16), dim3(block), 0, st, &p, sizeof(p));
        }
    });
    // X16R / X16RV2 nonce search (x16r.hip, search mode): `count` headers from one 80-byte template
    // with nNonce = start + i; every header of the window runs the same 16 slots (`slots_of_steps`,
    // from the template's hashPrevBlock), one launch per step, then x16r_hits keeps the lowest index
    // whose hash is <= the target. order: `count` identity indices; offsets: 16 x 17 (device).
    m.def("launch_x16r_search", [](const std::vector<const Kernel*>& slots, const Kernel& hits, uintptr_t tmpl,
                                   uintptr_t state, uintptr_t order, uintptr_t offsets,
                                   const std::vector<int>& slots_of_steps, uint32_t start, uint32_t count, bool v2,
                                   const std::string& target_le, uintptr_t best, uintptr_t stream) {
        if (count == 0) return;
        if (slots.size() != 16 || slots_of_steps.size() != 16 || target_le.size() != 32)
            throw std::invalid_argument("16 slot kernels, 16 steps, 32-byte target");
        X16rStepParams p{};
        p.state = reinterpret_cast<uint8_t*>(state);
        p.tmpl = reinterpret_cast<const uint8_t*>(tmpl);
        p.start_nonce = start;
        p.v2_all = v2 ? 1u : 0u;
        p.n = count;
        const hipStream_t st = as_stream(stream);
        for (uint32_t s = 0; s < 16; ++s) {
            const int a = slots_of_steps[s];
            if (a < 0 || a > 15) throw std::invalid_argument("slot out of range");
            p.step = s;
            p.order = reinterpret_cast<const int32_t*>(order);
            p.offsets = reinterpret_cast<const int32_t*>(offsets) + size_t(s) * 17;
            const unsigned block = unsigned(slots[size_t(a)]->max_threads);
            slots[size_t(a)]->launch_bytes(dim3((count + block - 1) / block), dim3(block), 0, st, &p, sizeof(p));
        }
        X16rHitParams h{};
        h.state = reinterpret_cast<const uint8_t*>(state);
        h.best = reinterpret_cast<uint32_t*>(best);
        std::memcpy(h.target, target_le.data(), 32);
        h.n = count;
        hits.launch_bytes(dim3((count + 255) / 256), dim3(256), 0, st, &h, sizeof(h));
    });
    m.def("sizeof_verify_job", [] { return sizeof(KawpowVerifyJob); });
    m.attr("KV_PROG_WORDS") = KV_PROG_WORDS;
    m.def("launch_kawpow_verify_light", [](const Kernel& k, uintptr_t light, uint32_t light_items, uintptr_t l1,
                                           uint32_t dag_items2048, uintptr_t jobs, uintptr_t programs,
                                           uint32_t num_programs, uintptr_t job_program, uint32_t num_jobs,
                                           uintptr_t out, uintptr_t stream) {
        if (num_programs == 0) throw std::invalid_argument("no programs");
        KawpowLightParams p{};
        p.light = reinterpret_cast<const void*>(light);
        p.l1 = reinterpret_cast<const uint32_t*>(l1);
        p.jobs = reinterpret_cast<const KawpowVerifyJob*>(jobs);
        p.programs = reinterpret_cast<const uint32_t*>(programs);
        p.job_program = reinterpret_cast<const uint32_t*>(job_program);
        p.out = reinterpret_cast<uint32_t*>(out);
        p.num_jobs = num_jobs;
        p.num_programs = num_programs;
        p.light_items = make_fastmod(light_items);
        p.items = make_fastmod(dag_items2048);
        const unsigned groups = 256 / 16;  // one job per 16-lane group (KL_BLOCK / 16)
        const unsigned grid = (num_jobs + groups - 1) / groups;
        if (grid == 0) return;
        k.launch_bytes(dim3(grid), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });
    m.def("launch_kawpow_verify_dag", [](const Kernel& k, uintptr_t dag, uint32_t dag_items2048, uintptr_t l1,
                                         uintptr_t jobs, uintptr_t programs, uint32_t num_programs,
                                         uintptr_t job_program, uint32_t num_jobs, uintptr_t out, uintptr_t stream) {
        if (num_programs == 0) throw std::invalid_argument("no programs");
        if (dag == 0) throw std::invalid_argument("kawpow_verify_dag needs a resident DAG");
        KawpowLightParams p{};
        p.dag = reinterpret_cast<const void*>(dag);
        p.l1 = reinterpret_cast<const uint32_t*>(l1);
        p.jobs = reinterpret_cast<const KawpowVerifyJob*>(jobs);
        p.programs = reinterpret_cast<const uint32_t*>(programs);
        p.job_program = reinterpret_cast<const uint32_t*>(job_program);
        p.out = reinterpret_cast<uint32_t*>(out);
        p.num_jobs = num_jobs;
        p.num_programs = num_programs;
        p.items = make_fastmod(dag_items2048);  // light_items unused in DAG mode
        const unsigned groups = 256 / 16;  // one job per 16-lane group
        const unsigned grid = (num_jobs + groups - 1) / groups;
        if (grid == 0) return;
        k.launch_bytes(dim3(grid), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });
    // kawpow_verify_waves: `slots` holds num_slots job indices (-1 = idle), 4 per wave, one period
    // per wave (ops/header_batch.py builds them); 4 waves per 256-thread workgroup
    m.def("launch_kawpow_verify_waves", [](const Kernel& k, uintptr_t dag, uint32_t dag_items2048, uintptr_t l1,
                                           uintptr_t jobs, uintptr_t programs, uint32_t num_programs,
                                           uintptr_t job_program, uint32_t num_jobs, uintptr_t slots,
                                           uint32_t num_slots, uintptr_t out, uintptr_t stream) {
        if (num_programs == 0) throw std::invalid_argument("no programs");
        if (dag == 0) throw std::invalid_argument("kawpow_verify_waves needs a resident DAG");
        if (num_slots % 4) throw std::invalid_argument("slots: 4 per wave");
        KawpowLightParams p{};
        p.dag = reinterpret_cast<const void*>(dag);
        p.l1 = reinterpret_cast<const uint32_t*>(l1);
        p.jobs = reinterpret_cast<const KawpowVerifyJob*>(jobs);
        p.programs = reinterpret_cast<const uint32_t*>(programs);
        p.job_program = reinterpret_cast<const uint32_t*>(job_program);
        p.out = reinterpret_cast<uint32_t*>(out);
        p.num_jobs = num_jobs;
        p.num_programs = num_programs;
        p.items = make_fastmod(dag_items2048);
        p.slots = reinterpret_cast<const int32_t*>(slots);
        p.num_slots = num_slots;
        const unsigned grid = (num_slots + 15) / 16;  // 16 slots (4 waves) per workgroup
        if (grid == 0) return;
        k.launch_bytes(dim3(grid), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });
    m.def("launch_kawpow_verify_batch", [](const Kernel& k, uintptr_t dag, uint32_t dag_items2048, uintptr_t jobs,
                                           uintptr_t programs, uintptr_t job_program, uint32_t num_jobs, uintptr_t out,
                                           uintptr_t stream) {
        if (num_jobs % 64) throw std::invalid_argument("verify batch must be padded to 64-job slabs");
        KawpowVerifyParams p{};
        p.dag = reinterpret_cast<const void*>(dag);
        p.jobs = reinterpret_cast<const KawpowVerifyJob*>(jobs);
        p.programs = reinterpret_cast<const uint32_t*>(programs);
        p.job_program = reinterpret_cast<const uint32_t*>(job_program);
        p.out = reinterpret_cast<uint32_t*>(out);
        p.num_jobs = num_jobs;
        p.items = make_fastmod(dag_items2048);
        const unsigned grid = (num_jobs + 255) / 256;
        if (grid == 0) return;
        k.launch_bytes(dim3(grid), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });

    // ---- batch ECDSA verification (secp256k1_verify.hip): n SecpVerifyJob records -> n u32 verdicts
    m.attr("SECP_JOB_BYTES") = sizeof(SecpVerifyJob);
    m.def("launch_secp_verify", [](const Kernel& k, uintptr_t jobs, uint32_t n, uintptr_t gtab, uintptr_t out,
                                   uintptr_t stream) {
        if (n == 0) return;
        SecpVerifyParams p{};
        p.jobs = reinterpret_cast<const SecpVerifyJob*>(jobs);
        p.gtab = reinterpret_cast<const uint32_t*>(gtab);
        p.out = reinterpret_cast<uint32_t*>(out);
        p.n = n;
        k.launch_bytes(dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });

    // ---- Equihash(200,9): one full Wagner solve for `num_inst` inputs, enqueued on `stream`
    m.attr("EQ_BUCKETS") = EQ_BUCKETS;
    m.attr("EQ_WORDS") = EQ_WORDS;
    m.attr("EQ_LEVELS") = EQ_LEVELS;
    m.attr("EQ_MAX_CAND") = EQ_MAX_CAND;
    m.attr("EQ_MAX_SOL") = EQ_MAX_SOL;
    m.attr("EQ_SOL_WORDS") = EQ_SOL_WORDS;
    // Batch SHA-256d (sha256d.hip): messages of `len` bytes at `stride`, or (merkle=true) one
    // ComputeMerkleRoot level of `len` 32-byte nodes into (len + 1) / 2 nodes.
    // header_batch.hip: hb_jobs / hb_verdict over rows [first, first + count) (`which` 0 / 1), or
    // hb_eq_scatter over the eq_n Equihash headers given (`which` 2)
    m.def("launch_header_batch", [](const Kernel& k, int which, uintptr_t rows, uintptr_t kinds, uintptr_t mixonly,
                                    uintptr_t jobs, uintptr_t job_program, uintptr_t full, uintptr_t out,
                                    uintptr_t eq_index, uintptr_t eq_verdict, uintptr_t eq_hash, uint32_t n,
                                    uint32_t eq_n, uint32_t first, uint32_t count, uint32_t epoch_length,
                                    int32_t last_checkpoint, const py::bytes& pow_limit_le, uintptr_t stream) {
        if (which < 2 && (first > n || count > n - first)) throw std::invalid_argument("row range outside the batch");
        if (epoch_length == 0 || epoch_length % 3) throw std::invalid_argument("epoch length must be a multiple of 3");
        const std::string lim = pow_limit_le;
        if (lim.size() != 32) throw std::invalid_argument("pow_limit must be 32 bytes");
        HeaderBatchParams p{};
        p.rows = reinterpret_cast<const uint8_t*>(rows);
        p.kinds = reinterpret_cast<const uint8_t*>(kinds);
        p.mixonly = reinterpret_cast<const uint8_t*>(mixonly);
        p.jobs = reinterpret_cast<KawpowVerifyJob*>(jobs);
        p.job_program = reinterpret_cast<uint32_t*>(job_program);
        p.full = reinterpret_cast<const uint32_t*>(full);
        p.out = reinterpret_cast<uint8_t*>(out);
        p.eq_index = reinterpret_cast<const uint32_t*>(eq_index);
        p.eq_verdict = reinterpret_cast<const uint32_t*>(eq_verdict);
        p.eq_hash = reinterpret_cast<const uint8_t*>(eq_hash);
        p.n = n;
        p.eq_n = eq_n;
        p.first = first;
        p.count = count;
        p.epoch_length = epoch_length;
        p.last_checkpoint = last_checkpoint;
        std::memcpy(p.pow_limit, lim.data(), 32);
        const uint32_t threads = which == 2 ? eq_n : count;
        if (threads == 0) return;
        k.launch_bytes(dim3((threads + 255) / 256), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });
    m.def("launch_kawpow_mixonly", [](const Kernel& k, uintptr_t headers, uint32_t n, uint32_t stride, uintptr_t out,
                                      uintptr_t stream) {
        if (stride < 120) throw std::invalid_argument("KawPow headers are 120 bytes");
        if (n == 0) return;
        MixOnlyParams p{};
        p.headers = reinterpret_cast<const uint8_t*>(headers);
        p.out = reinterpret_cast<uint8_t*>(out);
        p.n = n;
        p.stride = stride;
        k.launch_bytes(dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });
    m.def("launch_sha256d", [](const Kernel& k, uintptr_t in, uint32_t len, uint32_t stride, uint32_t n, uintptr_t out,
                               bool merkle, uintptr_t stream) {
        if (n == 0) return;
        if (merkle ? (n != (len + 1) / 2) : (len > stride || len > (1u << 24)))
            throw std::invalid_argument("bad sha256d geometry");
        Sha256dParams p{};
        p.in = reinterpret_cast<const uint8_t*>(in);
        p.out = reinterpret_cast<uint8_t*>(out);
        p.len = len;
        p.stride = stride;
        p.n = n;
        k.launch_bytes(dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });
    // Batch DarkGravityWave (dgw.hip): limits as 8 little-endian u32 limbs, compacts precomputed.
    m.def("launch_dgw", [](const Kernel& k, uintptr_t times, uintptr_t bits, uintptr_t out, uint32_t a, uint32_t n,
                           int32_t base_height, int32_t dgw_activation_block, uint32_t kawpow_time, uint32_t equihash_time,
                           std::vector<uint32_t> limits, std::vector<uint32_t> compacts, uint32_t target_timespan,
                           uintptr_t stream) {
        if (limits.size() != 24 || compacts.size() != 3) throw std::invalid_argument("3 limits of 8 limbs, 3 compacts");
        if (target_timespan == 0) throw std::invalid_argument("target_timespan must be positive");
        if (n == 0) return;
        DgwParams p{};
        p.times = reinterpret_cast<const uint32_t*>(times);
        p.bits = reinterpret_cast<const uint32_t*>(bits);
        p.out = reinterpret_cast<uint32_t*>(out);
        p.a = a;
        p.n = n;
        p.base_height = base_height;
        p.dgw_activation_block = dgw_activation_block;
        p.kawpow_time = kawpow_time;
        p.equihash_time = equihash_time;
        for (int i = 0; i < 8; ++i) {
            p.pow_limit[i] = limits[i];
            p.kawpow_limit[i] = limits[8 + i];
            p.equihash_limit[i] = limits[16 + i];
        }
        p.pow_limit_compact = compacts[0];
        p.kawpow_limit_compact = compacts[1];
        p.equihash_limit_compact = compacts[2];
        p.target_timespan = target_timespan;
        k.launch_bytes(dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });
    m.def("launch_equihash_verify", [](const Kernel& k, std::vector<uint64_t> h0, uintptr_t msgs, uint32_t input_len,
                                       uint32_t num, uintptr_t sols, uintptr_t out, uintptr_t stream) {
        if (h0.size() != 8) throw std::invalid_argument("h0 must have 8 words");
        if (input_len > 124) throw std::invalid_argument("equihash input must be <= 124 bytes");
        if (num == 0) return;
        EquihashVerifyParams p{};
        p.msgs = reinterpret_cast<const uint64_t*>(msgs);
        for (int i = 0; i < 8; ++i) p.h0[i] = h0[size_t(i)];
        p.input_len = input_len;
        p.num = num;
        p.sols = reinterpret_cast<const uint32_t*>(sols);
        p.out = reinterpret_cast<uint32_t*>(out);
        k.launch_bytes(dim3(num), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });
    m.attr("EQ_V_EMPTY") = EQ_V_EMPTY;
    m.def("launch_equihash_verify_slots", [](const Kernel& k, std::vector<uint64_t> h0, uintptr_t msgs,
                                             uint32_t input_len, uint32_t num_inst, uintptr_t sols, uintptr_t out,
                                             uintptr_t stream) {
        if (h0.size() != 8) throw std::invalid_argument("h0 must have 8 words");
        if (input_len > 124 || num_inst == 0 || num_inst > 65535) throw std::invalid_argument("bad equihash geometry");
        EquihashSlotVerifyParams p{};
        p.msgs = reinterpret_cast<const uint64_t*>(msgs);
        for (int i = 0; i < 8; ++i) p.h0[i] = h0[size_t(i)];
        p.input_len = input_len;
        p.num_inst = num_inst;
        p.sols = reinterpret_cast<const uint32_t*>(sols);
        p.out = reinterpret_cast<uint32_t*>(out);
        k.launch_bytes(dim3(EQ_MAX_SOL, num_inst), dim3(256), 0, as_stream(stream), &p, sizeof(p));
    });
    // Private-slot solver (equihash_ps.hip): ks = [eqp_gen, eqp_round1..8, eqp_final,
    // eqp_reconstruct]; `groups` workgroups per instance per round, EQP_SLOTS / groups rows per
    // segment. Buffers as documented on EquihashPsDev.
    m.attr("EQP_SLOTS") = EQP_SLOTS;
    m.attr("EQP_STAGE") = EQP_STAGE;
    m.attr("EQP_REF_STRIDE") = EQP_REF_STRIDE;
    m.attr("EQP_STATS") = EQP_STATS;
    m.attr("EQP_STAT_CHAIN") = EQP_STAT_CHAIN;
    m.attr("EQP_STAT_STAGE") = EQP_STAT_STAGE;
    m.attr("EQP_FINAL_GROUPS") = EQP_FINAL_GROUPS;
    m.attr("EQP_STAT_STAGE_MAX") = EQP_STAT_STAGE_MAX;
    m.def("launch_equihash_ps_solve", [](const std::vector<std::shared_ptr<Kernel>>& ks, std::vector<uint64_t> h0,
                                         uintptr_t msgs, uint32_t input_len, uint32_t num_inst, uint32_t groups,
                                         uintptr_t hashes, uintptr_t refs, uintptr_t counts, uintptr_t cands,
                                         uintptr_t sols, uintptr_t stats, uintptr_t stream, uint32_t block,
                                         uint32_t final_groups) {
        if (ks.size() != 11) throw std::invalid_argument("expected 11 equihash_ps kernels");
        if (final_groups == 0 || final_groups > EQ_BUCKETS) throw std::invalid_argument("final_groups: 1..4096");
        if (block < 256 || block > 1024 || block % 256) throw std::invalid_argument("block: 256..1024, a multiple of 256 (the build's EQP_BLOCK)");
        if (h0.size() != 8) throw std::invalid_argument("h0 must have 8 words");
        if (input_len > 124 || num_inst == 0 || num_inst > 65535) throw std::invalid_argument("bad equihash geometry");
        // P a power of two in [16, 256]: C = EQP_SLOTS / P fits the u8 counts and P the one-wave scan
        if (groups < 16 || groups > 256 || (groups & (groups - 1))) throw std::invalid_argument("groups: 16..256, 2^k");
        EquihashPsDev p{};
        p.msgs = reinterpret_cast<const uint64_t*>(msgs);
        for (int i = 0; i < 8; ++i) p.h0[i] = h0[size_t(i)];
        p.input_len = input_len;
        p.num_inst = num_inst;
        p.groups = groups;
        p.seg = EQP_SLOTS / groups;
        p.hashes = reinterpret_cast<uint32_t*>(hashes);
        p.refs = reinterpret_cast<uint32_t*>(refs);
        p.counts = reinterpret_cast<uint8_t*>(counts);
        p.cands = reinterpret_cast<uint32_t*>(cands);
        p.sols = reinterpret_cast<uint32_t*>(sols);
        p.stats = reinterpret_cast<uint32_t*>(stats);
        hipStream_t s = as_stream(stream);
        const size_t n = num_inst;
        check(hipMemsetAsync(p.cands, 0, n * (1 + 2 * EQ_MAX_CAND) * 4, s), "memset cands");
        check(hipMemsetAsync(p.sols, 0, n * (1 + EQ_MAX_SOL * 512) * 4, s), "memset sols");
        check(hipMemsetAsync(p.stats, 0, n * EQP_STATS * 4, s), "memset stats");
        // counts need no clear: every workgroup writes its whole row of every level
        const dim3 grid(groups, num_inst);
        for (size_t k = 0; k < 9; ++k) ks[k]->launch_bytes(grid, dim3(block), 0, s, &p, sizeof(p));
        ks[9]->launch_bytes(dim3(final_groups, num_inst), dim3(block), 0, s, &p, sizeof(p));
        ks[10]->launch_bytes(dim3(EQ_RECON_GROUPS, num_inst), dim3(256), 0, s, &p, sizeof(p));
    }, py::arg("ks"), py::arg("h0"), py::arg("msgs"), py::arg("input_len"), py::arg("num_inst"), py::arg("groups"),
       py::arg("hashes"), py::arg("refs"), py::arg("counts"), py::arg("cands"), py::arg("sols"), py::arg("stats"),
       py::arg("stream"), py::arg("block") = 1024, py::arg("final_groups") = EQP_FINAL_GROUPS);
}

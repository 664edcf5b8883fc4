// pybind11 module `parameter_server_distributed_amd._C`.
#include <torch/extension.h>

#include "async_hyper.h"
#include "async_ps.h"
#include "checkpoint.h"
#include "comm.h"
#include "kernels/launchers.h"
#include "kernels/launchers_gemm.h"
#include "ops.h"
#include "ps_core.h"
#include "registry.h"
#include "staleness.h"

namespace py = pybind11;
using namespace psd;

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X-native parameter-server runtime: gfx950 HIP kernels, RCCL comm, PS/coordinator cores";

  // ---- kernels ----
  m.def("fused_apply_", &fused_apply_, py::arg("master"), py::arg("grads"), py::arg("state1"), py::arg("state2"),
        py::arg("shadow"), py::arg("dyn"), py::arg("kind"), py::arg("momentum") = 0.0, py::arg("dampening") = 0.0,
        py::arg("nesterov") = false, py::arg("weight_decay") = 0.0, py::arg("beta1") = 0.9, py::arg("beta2") = 0.999,
        py::arg("eps") = 1e-8, py::arg("maximize") = false,
        py::arg("grid_cap") = 0);
  m.def(
      "async_hyper",
      [](int kind, int workers, double momentum, double beta1, double beta2, double weight_decay) {
        const AsyncHyper h = async_hyper(kind, workers, momentum, beta1, beta2, weight_decay);
        py::dict d;
        d["lr_factor"] = h.lr_factor;
        d["grad_scale"] = h.grad_scale;
        d["momentum"] = h.momentum;
        d["beta1"] = h.beta1;
        d["beta2"] = h.beta2;
        d["weight_decay"] = h.weight_decay;
        return d;
      },
      py::arg("kind"), py::arg("workers"), py::arg("momentum"), py::arg("beta1"), py::arg("beta2"),
      py::arg("weight_decay"), "per-push optimizer hyperparameters of an apply-on-arrival PS (async_hyper.h)");
  m.def("optim_advance_", &optim_advance_, py::arg("dyn"), py::arg("beta1") = 0.9, py::arg("beta2") = 0.999);
  m.def("multi_reduce_", &multi_reduce_, py::arg("out"), py::arg("srcs"), py::arg("scale") = 1.0);
  m.def("pack_cast_", &pack_cast_, py::arg("srcs"), py::arg("dsts"));
  m.def("xfer_", &xfer_, py::arg("srcs"), py::arg("dsts"), py::arg("blocks_per_seg"), py::arg("nt_store") = false);
  m.def("amax_", &amax_);
  m.def("quant_fp8_", &quant_fp8_);
  m.def("dequant_fp8_", &dequant_fp8_);
  m.def("quant_mx_", &quant_mx_, py::arg("x"), py::arg("out"), py::arg("scales"));
  m.def("dequant_mx_", &dequant_mx_, py::arg("q"), py::arg("scales"), py::arg("out"));
  m.def("quant_fp8_jit_", &quant_fp8_jit_, py::arg("x"), py::arg("out"), py::arg("scale_inv"));
  m.def("quant_fp8_delayed_", &quant_fp8_delayed_, py::arg("x"), py::arg("out"), py::arg("scale_inv"),
        py::arg("hist"), py::arg("margin") = 1.0);
  m.def("embed_bwd_", &embed_bwd_, py::arg("sorted"), py::arg("perm"), py::arg("dy"), py::arg("out"));
  m.def("xent_fwd", &xent_fwd, py::arg("x"), py::arg("labels"));
  m.def("xent_bwd", &xent_bwd, py::arg("x"), py::arg("labels"), py::arg("lse"), py::arg("scale"));
  m.def("bn_fwd", &bn_fwd, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("residual"), py::arg("relu"), py::arg("training"), py::arg("momentum"),
        py::arg("eps"), py::arg("counter"), py::arg("ss_eval"), py::arg("mask_out") = false,
        py::arg("residual_ss") = py::none(), py::arg("stats_only") = false, py::arg("q8_out") = py::none(),
        py::arg("part_in") = py::none(), py::arg("part_rows") = 0, py::arg("q8_mx") = py::none());
  m.def("bn_reduce_", &bn_reduce_, py::arg("x"), py::arg("shift"));
  m.def("bn_bwd_reduce_", &bn_bwd_reduce_, py::arg("dy"), py::arg("x"), py::arg("save_mean"),
        py::arg("ss") = py::none(), py::arg("dy2") = py::none(), py::arg("mbits") = py::none());
  m.def("bn_bwd_dual", &bn_bwd_dual, py::arg("dy"), py::arg("x"), py::arg("gamma"), py::arg("save_mean"),
        py::arg("save_invstd"), py::arg("mbits"), py::arg("dy2"), py::arg("xd"), py::arg("gamma_d"), py::arg("mean_d"),
        py::arg("invstd_d"), py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(),
        py::arg("dgamma_d_out") = py::none(), py::arg("dbeta_d_out") = py::none(), py::arg("fold") = false);
  m.def("bn_bwd_coef", &bn_bwd_coef, py::arg("dy"), py::arg("x"), py::arg("gamma"), py::arg("save_mean"),
        py::arg("save_invstd"), py::arg("mbits") = py::none(), py::arg("dy2") = py::none(), py::arg("part") = py::none(),
        py::arg("rows") = 0, py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none());
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("x"), py::arg("y"), py::arg("gamma"), py::arg("save_mean"),
        py::arg("save_invstd"), py::arg("relu"), py::arg("need_dr"), py::arg("dgamma_out"), py::arg("dbeta_out"),
        py::arg("dy2") = py::none(), py::arg("ss") = py::none(), py::arg("mbits") = py::none(),
        py::arg("dq") = py::none(), py::arg("dqmx") = py::none());
  m.def("gemm_", &gemm_, py::arg("A"), py::arg("B"), py::arg("a_kmajor"), py::arg("b_kmajor"), py::arg("out"),
        py::arg("bias") = py::none(), py::arg("act") = 0, py::arg("aux") = py::none(), py::arg("part") = py::none(),
        py::arg("shift") = py::none());
  m.def("gemm_stats_rows", &gemm_stats_rows_, py::arg("M"));
  m.def("gemm_set_bcontig", &gemm_set_bcontig, py::arg("on"));
  m.def("gemm_ct_", &gemm_ct_, py::arg("A"), py::arg("B"), py::arg("out"), py::arg("bias") = py::none(),
        py::arg("act") = 0, py::arg("aux") = py::none());
  m.def("gemm_gelu_bwd_", &gemm_gelu_bwd_, py::arg("A"), py::arg("B"), py::arg("a_kmajor"), py::arg("b_kmajor"),
        py::arg("pre"), py::arg("out"), py::arg("db"), py::arg("accumulate") = false);
  m.def("gemm_splitk_", &gemm_splitk_, py::arg("A"), py::arg("B"), py::arg("a_kmajor"), py::arg("b_kmajor"),
        py::arg("out"), py::arg("accumulate") = false, py::arg("scale") = 1.0, py::arg("splits") = 0);
  m.def("gemm_fp8_", &gemm_fp8_, py::arg("A"), py::arg("B"), py::arg("a_scale"), py::arg("b_scale"), py::arg("out"),
        py::arg("bias") = py::none(), py::arg("act") = 0, py::arg("aux") = py::none(), py::arg("part") = py::none(),
        py::arg("shift") = py::none());
  m.def("convn_", &convn_, py::arg("x"), py::arg("w2"), py::arg("out"), py::arg("R"), py::arg("S"), py::arg("stride"),
        py::arg("pad"), py::arg("part") = py::none(), py::arg("shift") = py::none(), py::arg("variant") = -1,
        py::arg("x2") = py::none(), py::arg("bias") = py::none(), py::arg("no_store") = false,
        py::arg("apply_ss") = py::none(), py::arg("apply_res") = py::none(), py::arg("apply_mask") = py::none());
  m.def("convn_stats_rows", &convn_stats_rows_, py::arg("M"));
  m.def("convn_part_rows", &convn_part_rows_, py::arg("M"), py::arg("N"), py::arg("variant"), py::arg("Ho"),
        py::arg("Wo"), py::arg("R"));
  m.def("convn_variant_ok", &convn_variant_ok_, py::arg("N"), py::arg("variant"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("Wo"), py::arg("has_x2") = false);
  m.def("convn_dgrad_s2_", &convn_dgrad_s2_, py::arg("dy"), py::arg("wph"), py::arg("out"), py::arg("variant"),
        py::arg("part") = py::none(), py::arg("bx") = py::none(), py::arg("bmean") = py::none(),
        py::arg("bss") = py::none());
  m.def("convn_dgrad_s2_rows", &convn_dgrad_s2_rows, py::arg("Nb"), py::arg("Ho"), py::arg("Wo"), py::arg("Ci"),
        py::arg("variant"));
  m.def("convn_bwd_", &convn_bwd_, py::arg("dy"), py::arg("w2"), py::arg("out"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("part"), py::arg("variant"), py::arg("mode"), py::arg("bx"),
        py::arg("bmean"), py::arg("bss") = py::none(), py::arg("bdr") = py::none(), py::arg("bmbits") = py::none(),
        py::arg("x2") = py::none(), py::arg("bias") = py::none(), py::arg("bxd") = py::none(),
        py::arg("bmean_d") = py::none(), py::arg("part_d") = py::none());
  m.def("bn_bwd_pre", &bn_bwd_pre, py::arg("g"), py::arg("x"), py::arg("gamma"), py::arg("save_mean"),
        py::arg("save_invstd"), py::arg("part"), py::arg("rows"), py::arg("dgamma_out") = py::none(),
        py::arg("dbeta_out") = py::none(), py::arg("dq") = py::none(), py::arg("dqmx") = py::none());
  m.def("convn_variants", &convn_variants_, py::arg("N"));
  m.def("convn_variant_kind", &convn_variant_kind_, py::arg("N"), py::arg("variant"));
  m.def("conv_fwd_", &conv_fwd_, py::arg("x"), py::arg("w2"), py::arg("out"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("part") = py::none(), py::arg("shift") = py::none());
  m.def("conv_wgrad_", &conv_wgrad_, py::arg("dy"), py::arg("x"), py::arg("out"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("splits") = 0);
  m.def("convw_", &convw_, py::arg("dy"), py::arg("x"), py::arg("out"), py::arg("R"), py::arg("S"), py::arg("stride"),
        py::arg("pad"), py::arg("variant") = -1, py::arg("accumulate") = false, py::arg("fold") = false);
  m.def("bn_bwd_dual_pre", &bn_bwd_dual_pre, py::arg("g"), py::arg("x"), py::arg("gamma"), py::arg("save_mean"),
        py::arg("save_invstd"), py::arg("part"), py::arg("part_d"), py::arg("rows"), py::arg("xd"), py::arg("gamma_d"),
        py::arg("mean_d"), py::arg("invstd_d"), py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(),
        py::arg("dgamma_d_out") = py::none(), py::arg("dbeta_d_out") = py::none(), py::arg("fold") = false,
        py::arg("fold_d") = false, py::arg("derive_d") = false);
  m.def("bn_elemt_coef", &bn_elemt_coef, py::arg("g"), py::arg("x"), py::arg("coef"));
  m.def("convw_fold_rows", &convw_fold_rows, py::arg("Cout"), py::arg("Cin"));
  m.def("convw_gram_rows", &convw_gram_rows_, py::arg("C"));
  m.def("convw_gram_", &convw_gram_, py::arg("x"), py::arg("out"), py::arg("variant") = 0);
  m.def("bnfold_dgrad_weights", &bnfold_dgrad_weights, py::arg("w"), py::arg("coef"));
  m.def("bnfold_rowdot", &bnfold_rowdot, py::arg("P"), py::arg("w"), py::arg("row"));
  m.def("bnfold_gram_stats", &bnfold_gram_stats, py::arg("P"), py::arg("w"), py::arg("shift"), py::arg("M"),
        py::arg("row"));
  m.def("bnfold_dual_weights", &bnfold_dual_weights, py::arg("w3"), py::arg("wd"), py::arg("ss3"), py::arg("ssd"));
  m.def("bn_finalize", &bn_finalize, py::arg("part"), py::arg("rows"), py::arg("M"), py::arg("gamma"),
        py::arg("beta"), py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"), py::arg("eps"),
        py::arg("counter") = py::none());
  m.def("bnfold_combine", &bnfold_combine, py::arg("P"), py::arg("w"), py::arg("coef"), py::arg("out"),
        py::arg("accumulate") = false);
  m.def("convw_variants", &convw_variants_, py::arg("Cout"), py::arg("KK"));
  m.def("conv_fwd_fp8_", &conv_fwd_fp8_, py::arg("x"), py::arg("w2"), py::arg("x_scale"), py::arg("w_scale"),
        py::arg("out"), py::arg("R"), py::arg("S"), py::arg("stride"), py::arg("pad"), py::arg("part") = py::none(),
        py::arg("shift") = py::none());
  m.def("gelu_bwd_colsum_", &gelu_bwd_colsum_, py::arg("dy"), py::arg("pre"), py::arg("dx"), py::arg("out"),
        py::arg("accumulate") = false);
  m.def("colsum_", &colsum_, py::arg("x"), py::arg("out"), py::arg("accumulate") = false);
  m.def("maxpool3s2_fwd", &maxpool3s2_fwd);
  m.def("maxpool3s2_bwd", &maxpool3s2_bwd, py::arg("dy"), py::arg("arg"), py::arg("H"), py::arg("W"),
        py::arg("dy2") = py::none());
  m.def("gap_fwd", &gap_fwd);
  m.def("bn_pool_fwd", &bn_pool_fwd, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("momentum"), py::arg("eps"), py::arg("counter") = py::none());
  m.def("stem_fwd", &stem_fwd, py::arg("x"), py::arg("w"), py::arg("gamma"), py::arg("beta"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("momentum"), py::arg("eps"), py::arg("counter") = py::none());
  m.def("stem_wgrad", &stem_wgrad);
  m.def("attn_fwd", &attn_fwd, py::arg("qkv"), py::arg("heads"), py::arg("p"), py::arg("seed"),
        py::arg("step") = py::none());
  m.def("attn_bwd", &attn_bwd, py::arg("dout"), py::arg("qkv"), py::arg("o"), py::arg("lse"), py::arg("heads"),
        py::arg("p"), py::arg("seed"), py::arg("step") = py::none(), py::arg("bias_out") = py::none());
  m.def("ln_fwd", &ln_fwd, py::arg("x"), py::arg("h"), py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("p"),
        py::arg("seed"), py::arg("step") = py::none());
  m.def("ln_bwd", &ln_bwd, py::arg("dy"), py::arg("s"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"), py::arg("p"),
        py::arg("seed"), py::arg("step") = py::none(), py::arg("dgamma_out") = py::none(),
        py::arg("dbeta_out") = py::none(), py::arg("dhsum_out") = py::none());
  m.def("emb_ln_fwd", &emb_ln_fwd, py::arg("ids"), py::arg("types"), py::arg("W"), py::arg("P"), py::arg("T"),
        py::arg("gamma"), py::arg("beta"), py::arg("S"), py::arg("eps"), py::arg("p"), py::arg("seed"),
        py::arg("step") = py::none());
  m.def("emb_ln_bwd", &emb_ln_bwd, py::arg("dy"), py::arg("ids"), py::arg("types"), py::arg("W"), py::arg("P"),
        py::arg("T"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"), py::arg("S"), py::arg("p"), py::arg("seed"),
        py::arg("step") = py::none(), py::arg("dgamma") = py::none(), py::arg("dbeta") = py::none(),
        py::arg("dT") = py::none());
  m.def("bn_pool_bwd", &bn_pool_bwd, py::arg("gpool"), py::arg("gpool2"), py::arg("arg"), py::arg("x"), py::arg("gamma"),
        py::arg("save_mean"), py::arg("save_invstd"), py::arg("ss"), py::arg("dgamma_out") = py::none(),
        py::arg("dbeta_out") = py::none());
  m.def("gap_bwd", &gap_bwd);
  m.def("subsample2", &subsample2, py::arg("x"));
  m.def("wprep_table", &wprep_table, py::arg("srcs"), py::arg("dsts"), py::arg("geo"));
  m.def("wprep_run", &wprep_run, py::arg("table"), py::arg("tiles"));
  m.attr("OPT_SGD") = (int)OPT_SGD;
  m.attr("OPT_MOMENTUM") = (int)OPT_MOMENTUM;
  m.attr("OPT_ADAM") = (int)OPT_ADAM;
  m.attr("OPT_ADAMW") = (int)OPT_ADAMW;

  // ---- checkpoint ----
  m.def("save_reference_ckpt", &save_reference_ckpt, py::call_guard<py::gil_scoped_release>());
  m.def("load_reference_ckpt", &load_reference_ckpt, py::call_guard<py::gil_scoped_release>());
  m.def("save_native_ckpt", &save_native_ckpt, py::call_guard<py::gil_scoped_release>());
  m.def("load_native_ckpt", &load_native_ckpt, py::call_guard<py::gil_scoped_release>());
  m.def("crc32", [](py::bytes b) {
    std::string s = b;
    return crc32(s.data(), s.size());
  });

  // ---- coordinator core ----
  py::class_<WorkerEntry>(m, "WorkerEntry")
      .def_readonly("worker_id", &WorkerEntry::worker_id)
      .def_readonly("address", &WorkerEntry::address)
      .def_readonly("port", &WorkerEntry::port)
      .def_readonly("hostname", &WorkerEntry::hostname)
      .def_readonly("status", &WorkerEntry::status)
      .def_readonly("last_heartbeat", &WorkerEntry::last_heartbeat)
      .def_readonly("join_epoch", &WorkerEntry::join_epoch);
  py::class_<RegisterResult>(m, "RegisterResult")
      .def_readonly("success", &RegisterResult::success)
      .def_readonly("message", &RegisterResult::message)
      .def_readonly("ps_address", &RegisterResult::ps_address)
      .def_readonly("total_workers", &RegisterResult::total_workers)
      .def_readonly("membership_epoch", &RegisterResult::membership_epoch);
  py::class_<ShardInfo>(m, "ShardInfo")
      .def_readonly("shard_id", &ShardInfo::shard_id)
      .def_readonly("address", &ShardInfo::address)
      .def_readonly("rank", &ShardInfo::rank);
  py::class_<Registry>(m, "Registry")
      .def(py::init<std::string, int32_t>())
      .def("register_worker", &Registry::register_worker)
      .def("heartbeat", &Registry::heartbeat)
      .def("deregister", &Registry::deregister)
      .def("list_workers", &Registry::list_workers)
      .def("live_ids", &Registry::live_ids)
      .def("ps_address", &Registry::ps_address)
      .def("set_ps_address", &Registry::set_ps_address)
      .def("remove_stale", &Registry::remove_stale)
      .def("membership_epoch", &Registry::membership_epoch)
      .def("wait_epoch_change", &Registry::wait_epoch_change, py::call_guard<py::gil_scoped_release>())
      .def("set_shard", &Registry::set_shard)
      .def("shards", &Registry::shards)
      .def("kv_set", [](Registry& r, const std::string& k, py::bytes v) { r.kv_set(k, std::string(v)); })
      .def("kv_get",
           [](Registry& r, const std::string& k, double timeout) {
             std::tuple<bool, std::string> res;
             {
               py::gil_scoped_release nogil;
               res = r.kv_get(k, timeout);
             }
             return py::make_tuple(std::get<0>(res), py::bytes(std::get<1>(res)));
           })
      .def("use_manual_clock", &Registry::use_manual_clock)
      .def("advance_clock", &Registry::advance_clock)
      .def("now", &Registry::now);

  // ---- parameter-server core ----
  py::class_<PSConfig>(m, "PSConfig")
      .def(py::init<>())
      .def_readwrite("total_workers", &PSConfig::total_workers)
      .def_readwrite("async_mode", &PSConfig::async_mode)
      .def_readwrite("staleness_bound", &PSConfig::staleness_bound)
      .def_readwrite("window", &PSConfig::window)
      .def_readwrite("opt_kind", &PSConfig::opt_kind)
      .def_readwrite("lr", &PSConfig::lr)
      .def_readwrite("momentum", &PSConfig::momentum)
      .def_readwrite("dampening", &PSConfig::dampening)
      .def_readwrite("weight_decay", &PSConfig::weight_decay)
      .def_readwrite("beta1", &PSConfig::beta1)
      .def_readwrite("beta2", &PSConfig::beta2)
      .def_readwrite("eps", &PSConfig::eps)
      .def_readwrite("nesterov", &PSConfig::nesterov)
      .def_readwrite("reference_compat", &PSConfig::reference_compat)
      .def_readwrite("staleness_lr_scaling", &PSConfig::staleness_lr_scaling)
      .def_readwrite("async_grad_scale", &PSConfig::async_grad_scale)
      .def_readwrite("pull_timeout_s", &PSConfig::pull_timeout_s);
  py::class_<PushResult>(m, "PushResult")
      .def_readonly("success", &PushResult::success)
      .def_readonly("message", &PushResult::message)
      .def_readonly("iteration", &PushResult::iteration)
      .def_readonly("aggregation_complete", &PushResult::aggregation_complete)
      .def_readonly("workers_received", &PushResult::workers_received)
      .def_readonly("total_workers", &PushResult::total_workers)
      .def_readonly("version", &PushResult::version)
      .def_readonly("staleness", &PushResult::staleness);
  py::class_<PSCore>(m, "PSCore")
      .def(py::init<PSConfig, std::string>())
      .def("initialized", &PSCore::initialized)
      .def("init_params", &PSCore::init_params, py::call_guard<py::gil_scoped_release>())
      .def("names", &PSCore::names)
      .def("shapes", &PSCore::shapes)
      .def("offsets", &PSCore::offsets)
      .def("numel", &PSCore::numel)
      .def("push", &PSCore::push, py::call_guard<py::gil_scoped_release>())
      .def("pull", &PSCore::pull, py::call_guard<py::gil_scoped_release>())
      .def("sync_status", &PSCore::sync_status)
      .def("set_total_workers", &PSCore::set_total_workers, py::call_guard<py::gil_scoped_release>())
      .def("forget_worker", &PSCore::forget_worker)
      .def("total_workers", &PSCore::total_workers)
      .def("current_iteration", &PSCore::current_iteration)
      .def("version", &PSCore::version)
      .def("staleness_histogram", &PSCore::staleness_histogram)
      .def("counters", &PSCore::counters)
      .def("save_reference", &PSCore::save_reference, py::call_guard<py::gil_scoped_release>())
      .def("load_reference", &PSCore::load_reference, py::call_guard<py::gil_scoped_release>())
      .def("state_tensors", &PSCore::state_tensors)
      .def("load_state_tensors", &PSCore::load_state_tensors);

  // ---- staleness / version bookkeeping for the collective data plane ----
  py::class_<StalenessTracker>(m, "StalenessTracker")
      .def(py::init<int, int>(), py::arg("num_shards"), py::arg("bins") = 64)
      .def("on_pull", &StalenessTracker::on_pull)
      .def("on_apply", &StalenessTracker::on_apply)
      .def("version", &StalenessTracker::version)
      .def("histogram", &StalenessTracker::histogram)
      .def("percentile", &StalenessTracker::percentile)
      .def("reset", &StalenessTracker::reset);

  // ---- asynchronous apply-on-arrival PS over peer memory ----
  py::class_<AsyncEngine>(m, "AsyncEngine")
      .def(py::init<int, int, std::vector<int>, std::vector<int>, std::vector<int64_t>, std::vector<int64_t>, int, int,
                    std::string, bool, int, double, int, bool>(),
           py::arg("rank"), py::arg("world"), py::arg("owners"), py::arg("workers"), py::arg("shard_off"),
           py::arg("shard_len"), py::arg("staleness"), py::arg("nbuf"), py::arg("shm_name"), py::arg("create"),
           py::arg("device"), py::arg("timeout_s"), py::arg("elem_bytes") = 2, py::arg("mx") = false)
      .def("local_desc", [](const AsyncEngine& e) { return py::bytes(e.local_desc()); })
      .def("attach_peer", [](AsyncEngine& e, int r, py::bytes d) { e.attach_peer(r, std::string(d)); })
      .def("set_shard_state", &AsyncEngine::set_shard_state)
      .def("publish_initial", &AsyncEngine::publish_initial, py::arg("shard"), py::arg("version") = 0,
           py::arg("clocks") = std::vector<int64_t>{})
      .def("set_round", &AsyncEngine::set_round)
      .def("set_fixed_schedule", &AsyncEngine::set_fixed_schedule)
      .def("start", &AsyncEngine::start)
      .def("stop", &AsyncEngine::stop, py::call_guard<py::gil_scoped_release>())
      .def("close_peers", &AsyncEngine::close_peers)
      .def("free_local", &AsyncEngine::free_local)
      .def("pull", &AsyncEngine::pull, py::call_guard<py::gil_scoped_release>())
      .def("pull_mx", &AsyncEngine::pull_mx, py::call_guard<py::gil_scoped_release>())
      .def("push", &AsyncEngine::push, py::call_guard<py::gil_scoped_release>())
      .def("commit", &AsyncEngine::commit, py::call_guard<py::gil_scoped_release>())
      .def("wait_applied", &AsyncEngine::wait_applied, py::call_guard<py::gil_scoped_release>())
      .def("wait_all_applied", &AsyncEngine::wait_all_applied, py::call_guard<py::gil_scoped_release>())
      .def("inbox_view", &AsyncEngine::inbox_view)
      .def("histogram", &AsyncEngine::histogram)
      .def("version", &AsyncEngine::version)
      .def("clocks", &AsyncEngine::clocks)
      .def("my_shards", &AsyncEngine::my_shards)
      .def("memory_kind", &AsyncEngine::memory_kind)
      .def("set_xfer", &AsyncEngine::set_xfer)
      .def("xfer_mode", &AsyncEngine::xfer_mode)
      .def("set_xfer_blocks", &AsyncEngine::set_xfer_blocks)
      .def("xfer_blocks_cap", &AsyncEngine::xfer_blocks_cap)
      .def("error", &AsyncEngine::error)
      .def("inject_error", &AsyncEngine::inject_error)
      .def("counters", &AsyncEngine::counters)
      .def("enable_log", &AsyncEngine::enable_log)
      .def("apply_log", &AsyncEngine::apply_log);

  // ---- RCCL ----
  py::class_<RcclComm>(m, "RcclComm")
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def_static("version", &RcclComm::version)
      .def(py::init([](int rank, int world, py::bytes uid, int device) {
             std::string u = uid;
             py::gil_scoped_release nogil;
             return new RcclComm(rank, world, u, device);
           }),
           py::arg("rank"), py::arg("world"), py::arg("uid"), py::arg("device"))
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def("all_reduce", &RcclComm::all_reduce, py::arg("t"), py::arg("op") = "sum", py::arg("stream") = 0)
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::arg("inp"), py::arg("out"), py::arg("op") = "sum",
           py::arg("stream") = 0)
      .def("all_gather", &RcclComm::all_gather, py::arg("inp"), py::arg("out"), py::arg("stream") = 0)
      .def("reduce", &RcclComm::reduce, py::arg("inp"), py::arg("out"), py::arg("root"), py::arg("op") = "sum",
           py::arg("stream") = 0)
      .def("broadcast", &RcclComm::broadcast, py::arg("t"), py::arg("root"), py::arg("stream") = 0)
      .def("send", &RcclComm::send, py::arg("t"), py::arg("peer"), py::arg("stream") = 0)
      .def("recv", &RcclComm::recv, py::arg("t"), py::arg("peer"), py::arg("stream") = 0)
      .def_static("group_start", &RcclComm::group_start)
      .def_static("group_end", &RcclComm::group_end)
      .def("abort", &RcclComm::abort)
      .def("async_error", &RcclComm::async_error);
}

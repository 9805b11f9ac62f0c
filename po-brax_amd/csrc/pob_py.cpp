// pob_py.cpp -- the pybind11 module `po_brax_amd._pob`: a thin binding of the C ABI
// (include/pob.h) for the per-step entry points, the ones the Python env layer calls on
// every env-step (pob_step, pob_reset_where_done_shard) or reset (pob_reset).
//
// Arguments are what the C ABI takes, as Python ints: env handles, device pointers
// (torch.Tensor.data_ptr()), addresses of pob_state structs (ctypes.addressof of the
// struct the env layer builds and caches) and hipStream_t handles (torch's
// current_stream().cuda_stream).  No torch types cross this boundary.  Status codes map to the
// reference's exception types: POB_EINVAL -> ValueError, anything else -> RuntimeError (the
// ctypes binding's PobError is a RuntimeError too), with pob_last_error()'s message.
// A pybind11 call costs well under a microsecond of host time; the ctypes call it replaces
// marshalled eight arguments per step through libffi.
//
// The module does not link libpob.so: `bind()` receives the entry points of the libpob.so the
// ctypes layer loaded (po_brax_amd._lib, which honours POB_LIB), so both bindings always call
// the same library -- an A/B run of another build never mixes two copies.
#include <pybind11/pybind11.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "../../include/pob.h"

namespace py = pybind11;

namespace {

using step_fn = decltype(&pob_step);
using reset_fn = decltype(&pob_reset);
using rwd_fn = decltype(&pob_reset_where_done_shard);
using err_fn = decltype(&pob_last_error);
step_fn g_step = nullptr;
reset_fn g_reset = nullptr;
rwd_fn g_rwd = nullptr;
err_fn g_err = nullptr;

void bound() {
  if (!g_step || !g_reset || !g_rwd || !g_err) throw std::runtime_error("_pob: bind() was not called");
}

void check(int rc) {
  if (rc == POB_OK) return;
  const char *m = g_err();
  const std::string msg = m ? m : "";
  if (rc == POB_EINVAL) throw py::value_error(msg);
  throw std::runtime_error("libpob status " + std::to_string(rc) + ": " + msg);
}

template <typename T>
T *P(std::uintptr_t a) { return reinterpret_cast<T *>(a); }

}  // namespace

PYBIND11_MODULE(_pob, m) {
  m.doc() = "pybind11 binding of libpob's per-step C ABI (include/pob.h)";
  m.def(
      "bind",
      [](std::uintptr_t step, std::uintptr_t reset, std::uintptr_t rwd, std::uintptr_t last_error) {
        g_step = reinterpret_cast<step_fn>(step);
        g_reset = reinterpret_cast<reset_fn>(reset);
        g_rwd = reinterpret_cast<rwd_fn>(rwd);
        g_err = reinterpret_cast<err_fn>(last_error);
      },
      py::arg("pob_step"), py::arg("pob_reset"), py::arg("pob_reset_where_done_shard"), py::arg("pob_last_error"));
  // pob_step(env, B, in, act, out, flags, episode_length, stream): in / out are pob_state
  // struct addresses (equal for an in-place step)
  m.def(
      "step",
      [](std::uintptr_t env, int B, std::uintptr_t in, std::uintptr_t act, std::uintptr_t out, std::uint32_t flags,
         int episode_length, std::uintptr_t stream) {
        bound();
        check(g_step(P<pob_env>(env), B, P<const pob_state>(in), P<const float>(act), P<const pob_state>(out),
                       flags, episode_length, P<void>(stream)));
      },
      py::arg("env"), py::arg("B"), py::arg("state_in"), py::arg("act"), py::arg("state_out"), py::arg("flags"),
      py::arg("episode_length"), py::arg("stream"));
  m.def(
      "reset",
      [](std::uintptr_t env, int B, std::uintptr_t keys, std::uintptr_t out, std::uintptr_t stream) {
        bound();
        check(g_reset(P<pob_env>(env), B, P<const std::uint32_t>(keys), P<const pob_state>(out), P<void>(stream)));
      },
      py::arg("env"), py::arg("B"), py::arg("keys"), py::arg("state"), py::arg("stream"));
  m.def(
      "reset_where_done_shard",
      [](std::uintptr_t env, int B, int total, int first, int mode, std::uintptr_t gym_in, std::uintptr_t gym_out,
         std::uintptr_t s, std::uintptr_t stream) {
        bound();
        check(g_rwd(P<pob_env>(env), B, total, first, mode, P<const std::uint32_t>(gym_in),
                                         P<std::uint32_t>(gym_out), P<const pob_state>(s), P<void>(stream)));
      },
      py::arg("env"), py::arg("B"), py::arg("total"), py::arg("first"), py::arg("mode"), py::arg("gym_in"),
      py::arg("gym_out"), py::arg("state"), py::arg("stream"));
  m.attr("ENTRY_POINTS") = py::make_tuple("pob_step", "pob_reset", "pob_reset_where_done_shard");
}

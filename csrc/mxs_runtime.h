// mxstream — host runtime (C++): string dictionary, Java-compatible text parsing, socket
// source, key-group-indexed checkpoint files.
#pragma once
#include <pybind11/pybind11.h>

void bind_runtime(pybind11::module_& m);
void bind_sessions(pybind11::module_& m);
void bind_vector(pybind11::module_& m);
void bind_trace(pybind11::module_& m);
void bind_check(pybind11::module_& m);
void bind_reader(pybind11::module_& m);
void bind_format(pybind11::module_& m);
void bind_listwin(pybind11::module_& m);
void bind_window_tier(pybind11::module_& m);
void bind_window_control(pybind11::module_& m);

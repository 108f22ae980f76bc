// rtow_internal.h — shared between the host and device halves of librtow_hip.so.
#pragma once
#include <string>

// Record `msg` for rtow_last_error() and return `code`.
int set_error(int code, const std::string& msg);

// Host-side table utilities (mox_table.cpp); internal to libmox.so.
#pragma once
#include <stdint.h>

namespace mox_host {
// Bytewise ascending order (Rust String Ord) of a fetched table, in place.
// Returns 0, or -1 when a host allocation fails.
int sort_table_bytes(uint64_t n, uint64_t* counts, uint64_t* offs, uint8_t* bytes);
}  // namespace mox_host

/*
 * prismdb_synth.h -- synthetic SST-block generator on the device (bench and
 * test support; not part of the checksum path).
 *
 * Fills dev_dst[0, nbytes) with bytes [byte_offset, byte_offset + nbytes) of the
 * stream of little-endian u64 words word[k] = splitmix64(seed, k)
 * (z = seed + (k+1)*0x9E3779B97F4A7C15, then the splitmix64 finaliser).
 * byte_offset must be a multiple of 8 and dev_dst 16-byte aligned.
 * Returns 0 on success, < 0 on bad arguments or a launch error.
 */
#ifndef PRISMDB_SYNTH_H_
#define PRISMDB_SYNTH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int prismdb_fill_synthetic(void* dev_dst, size_t nbytes, uint64_t seed, uint64_t byte_offset,
                           void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PRISMDB_SYNTH_H_ */

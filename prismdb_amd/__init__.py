"""prismdb_amd -- MI355X-native block-checksum engine for PrismDB/LevelDB.

The one hot path built here is CRC32C over SST blocks (util/crc32c.cc,
table/table_builder.cc:185-202, table/format.cc:91-102), batched onto
hand-written gfx950 HIP kernels behind a C ABI (include/prismdb_crc32c.h).

Modules:
    prismdb_amd.crc32c   leveldb::crc32c surface (host) + device batch API
    prismdb_amd.sst      SST footer/index parsing and per-file batch verify
    prismdb_amd.dist     multi-GPU sharding with an RCCL gather of results
    prismdb_amd.build    in-tree hipcc build of the native library
"""

__all__ = ["crc32c"]

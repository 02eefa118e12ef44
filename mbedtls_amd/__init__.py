"""mbedtls_amd -- MI355X TLS record-layer AEAD engine.

A drop-in for the record encrypt/decrypt path of Mbed TLS 4.1.0
(``mbedtls_ssl_encrypt_buf`` / ``mbedtls_ssl_decrypt_buf``, library/ssl_msg.c)
with hand-written gfx950 kernels for AES-128/256-GCM and ChaCha20-Poly1305.
The C ABI is include/tlsrec.h; this package is its Python binding.
"""
from ._abi import (CIPHER_AES_128_GCM, CIPHER_AES_256_GCM, CIPHER_CHACHA20_POLY1305,  # noqa: F401
                   CIPHER_AES_192_GCM, CIPHER_AES_128_CCM, CIPHER_AES_192_CCM, CIPHER_AES_256_CCM,
                   CIPHER_AES_128_CCM_8, CIPHER_AES_192_CCM_8, CIPHER_AES_256_CCM_8, KEYLEN, TAGLEN,
                   CIPHER_ARIA_128_GCM, CIPHER_ARIA_192_GCM, CIPHER_ARIA_256_GCM,
                   CIPHER_ARIA_128_CCM, CIPHER_ARIA_192_CCM, CIPHER_ARIA_256_CCM,
                   CIPHER_CAMELLIA_128_GCM, CIPHER_CAMELLIA_192_GCM, CIPHER_CAMELLIA_256_GCM,
                   CIPHER_CAMELLIA_128_CCM, CIPHER_CAMELLIA_192_CCM, CIPHER_CAMELLIA_256_CCM,
                   ERR_SSL_BAD_INPUT_DATA, ERR_SSL_BUFFER_TOO_SMALL, ERR_SSL_FEATURE_UNAVAILABLE, ERR_SSL_ALLOC_FAILED,
                   ERR_SSL_HW_ACCEL_FAILED, ERR_SSL_INTERNAL_ERROR, ERR_SSL_INVALID_MAC,
                   ERR_SSL_INVALID_RECORD, ERR_SSL_UNEXPECTED_CID, MSG_APPLICATION_DATA, MSG_CID,
                   CID_LEN_MAX, VERSION_TLS1_2, VERSION_TLS1_3, ERR_SSL_COUNTER_WRAPPING,
                   ERR_SSL_UNEXPECTED_RECORD, ERR_SSL_EARLY_MESSAGE, ERR_SSL_CONN_EOF, DTLS_MAX_DATAGRAM,
                   DTLS_OUT_BUFFER_LEN, DTLS_DROPPED, DTLS_NOT_REACHED, DTLS_ANTI_REPLAY,
                   DTLS_IGNORE_UNEXPECTED_CID,
                   BATCH_REC, BATCH_RES, KEY_MATERIAL, load)
from .batch import (KeyTable, batch_decrypt, batch_encrypt, frame_check, host_batch, key_material,  # noqa: F401
                    records, results, seq_bytes)
from .record import Record, Transform, decrypt_buf, encrypt_buf  # noqa: F401
from .shard import Shard, broadcast_keys, reduce_status, shard_bounds, status_counts  # noqa: F401


def device_ok() -> bool:
    """True when a gfx950 device is usable by libtlsrec."""
    return load().tlsrec_device_check() == 0


def version() -> str:
    return load().tlsrec_version_string().decode()

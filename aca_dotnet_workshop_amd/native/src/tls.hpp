// TLS for the epoll HTTP stack (evhttp.hpp) over the system OpenSSL (libssl / libcrypto).
//
// Uses: HTTPS listeners (external ingress equivalent, `--app-ssl` app endpoints), and mutual
// TLS between sidecars (Dapr Sentry equivalent): every sidecar presents the workload
// certificate the environment CA issued for its app-id (platform/pki.py) and verifies the
// peer's -- a client checks the server certificate names the app-id it meant to call, a
// server requires a client certificate from the same CA.
//
// Non-blocking operation on level-triggered epoll: `TlsIo::recv/send` map OpenSSL's
// WANT_READ / WANT_WRITE onto EAGAIN (with `want_write` telling the connection to also poll
// for writability); the handshake is driven implicitly by the first reads / writes.
// Session tickets are off (TLS 1.3 tickets would be written from inside SSL_read).
#pragma once

#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <arpa/inet.h>

#include <atomic>
#include <cerrno>
#include <memory>
#include <stdexcept>
#include <string>
#include <sys/types.h>

namespace tt::ev {

struct TlsConfig {
  std::string cert, key, ca;
  bool verify_peer = true;  // server: require a client certificate (mutual TLS); client: verify the server
};

// Server-side handshakes refused (no client certificate, one from another CA, a protocol
// error before the handshake finished): the data plane's evidence that mTLS turned a peer away
// (`sidecar_mtls_handshake_rejected_total` on its /metrics), independent of how the refused
// client happened to report it.
inline std::atomic<uint64_t> tls_server_handshake_rejects{0};

inline std::string tls_error_text() {
  unsigned long e = ERR_get_error();
  char buf[256];
  ERR_error_string_n(e, buf, sizeof buf);
  return buf;
}

class TlsContext {
 public:
  TlsContext(const TlsConfig& cfg, bool server) : server_(server) {
    ctx_ = SSL_CTX_new(server ? TLS_server_method() : TLS_client_method());
    if (!ctx_) throw std::runtime_error("SSL_CTX_new: " + tls_error_text());
    SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
    SSL_CTX_set_mode(ctx_, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
    SSL_CTX_set_options(ctx_, SSL_OP_NO_TICKET);
    SSL_CTX_set_num_tickets(ctx_, 0);
    // one read(2) per readiness instead of two per record (5-byte header, then the body):
    // OpenSSL buffers what arrived, and `pending()` reports that buffer (SSL_has_pending), so
    // the readers keep going until it is empty -- epoll would not wake them for it
    SSL_CTX_set_read_ahead(ctx_, 1);
    if (!cfg.cert.empty()) {
      if (SSL_CTX_use_certificate_chain_file(ctx_, cfg.cert.c_str()) != 1 ||
          SSL_CTX_use_PrivateKey_file(ctx_, cfg.key.c_str(), SSL_FILETYPE_PEM) != 1)
        throw std::runtime_error("TLS certificate " + cfg.cert + ": " + tls_error_text());
    }
    if (cfg.verify_peer) {
      if (cfg.ca.empty() || SSL_CTX_load_verify_locations(ctx_, cfg.ca.c_str(), nullptr) != 1)
        throw std::runtime_error("TLS CA " + cfg.ca + ": " + tls_error_text());
      SSL_CTX_set_verify(ctx_, server ? (SSL_VERIFY_PEER | SSL_VERIFY_FAIL_IF_NO_PEER_CERT) : SSL_VERIFY_PEER,
                         nullptr);
    } else {
      SSL_CTX_set_verify(ctx_, SSL_VERIFY_NONE, nullptr);  // `--app-ssl`: the app's dev certificate
    }
  }
  ~TlsContext() { SSL_CTX_free(ctx_); }
  TlsContext(const TlsContext&) = delete;
  TlsContext& operator=(const TlsContext&) = delete;
  SSL_CTX* get() const { return ctx_; }
  bool server() const { return server_; }

 private:
  SSL_CTX* ctx_ = nullptr;
  bool server_;
};

class TlsIo {
 public:
  // `peer_name`: client side -- the name the server certificate must carry (empty: any).
  TlsIo(const TlsContext& ctx, int fd, const std::string& peer_name = "") {
    ssl_ = SSL_new(ctx.get());
    if (!ssl_) throw std::runtime_error("SSL_new: " + tls_error_text());
    SSL_set_fd(ssl_, fd);
    if (ctx.server()) {
      SSL_set_accept_state(ssl_);
    } else {
      SSL_set_connect_state(ssl_);
      if (!peer_name.empty()) {
        in_addr a4{};
        if (inet_pton(AF_INET, peer_name.c_str(), &a4) == 1) {
          // an address, as a browser typed it: checked against the certificate's IP SANs (no SNI)
          X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(ssl_), peer_name.c_str());
        } else {
          SSL_set_tlsext_host_name(ssl_, peer_name.c_str());
          SSL_set_hostflags(ssl_, X509_CHECK_FLAG_NO_PARTIAL_WILDCARDS);
          SSL_set1_host(ssl_, peer_name.c_str());
        }
      }
    }
  }
  ~TlsIo() {
    if (ssl_) SSL_free(ssl_);
  }
  TlsIo(const TlsIo&) = delete;
  TlsIo& operator=(const TlsIo&) = delete;

  // recv(2)/send(2) semantics: > 0 bytes, 0 = orderly close, -1 with errno (EAGAIN: retry on
  // readiness -- poll for writability too while `want_write`).
  ssize_t recv(char* buf, size_t n) {
    ERR_clear_error();
    int r = SSL_read(ssl_, buf, (int)std::min<size_t>(n, 1 << 30));
    if (r > 0) {
      want_write = false;
      return r;
    }
    return fail(r);
  }
  ssize_t send(const char* p, size_t n) {
    ERR_clear_error();
    int r = SSL_write(ssl_, p, (int)std::min<size_t>(n, 1 << 30));
    if (r > 0) {
      want_write = false;
      return r;
    }
    return fail(r);
  }
  // decrypted bytes not yet returned, or raw bytes read ahead and not yet processed
  bool pending() const { return SSL_has_pending(ssl_) == 1; }
  // Names (SAN DNS / URI entries) in the verified peer certificate; empty without one.
  std::string peer_names() const {
    std::string out;
    X509* c = SSL_get1_peer_certificate(ssl_);
    if (!c) return out;
    auto* names = (GENERAL_NAMES*)X509_get_ext_d2i(c, NID_subject_alt_name, nullptr, nullptr);
    for (int i = 0; names && i < sk_GENERAL_NAME_num(names); ++i) {
      const GENERAL_NAME* g = sk_GENERAL_NAME_value(names, i);
      if (g->type != GEN_DNS && g->type != GEN_URI) continue;
      const ASN1_IA5STRING* s = g->type == GEN_DNS ? g->d.dNSName : g->d.uniformResourceIdentifier;
      if (!out.empty()) out += ',';
      out.append((const char*)ASN1_STRING_get0_data(s), (size_t)ASN1_STRING_length(s));
    }
    GENERAL_NAMES_free(names);
    X509_free(c);
    return out;
  }
  bool want_write = false;
  std::string last_error;

 private:
  SSL* ssl_ = nullptr;

  ssize_t fail(int r) {
    int e = SSL_get_error(ssl_, r);
    switch (e) {
      case SSL_ERROR_WANT_READ:
        want_write = false;
        errno = EAGAIN;
        return -1;
      case SSL_ERROR_WANT_WRITE:
        want_write = true;
        errno = EAGAIN;
        return -1;
      case SSL_ERROR_ZERO_RETURN:
        return 0;
      case SSL_ERROR_SYSCALL:
        if (errno == 0 || errno == EAGAIN) return errno == EAGAIN ? (errno = EAGAIN, -1) : 0;
        return -1;
      default:
        last_error = tls_error_text();
        if (SSL_is_server(ssl_) && !SSL_is_init_finished(ssl_))
          tls_server_handshake_rejects.fetch_add(1, std::memory_order_relaxed);
        errno = ECONNRESET;  // handshake / verification failure or a corrupt record
        return -1;
    }
  }
};

}  // namespace tt::ev

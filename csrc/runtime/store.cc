// TCP key-value store: the rendezvous server hosted by `mihvdrun` and the
// control channel of the negotiation engine (negotiator.cc). One poll() thread serves every
// connection; blocking reads are parked as waiters and answered when their keys appear or their
// deadline passes.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>

#include "control.h"

namespace mihvd {

namespace {

using Clock = std::chrono::steady_clock;

void put_u32(std::string& s, uint32_t v) {
  char b[4];
  std::memcpy(b, &v, 4);
  s.append(b, 4);
}
void put_i64(std::string& s, int64_t v) {
  char b[8];
  std::memcpy(b, &v, 8);
  s.append(b, 8);
}
void put_str(std::string& s, const std::string& v) {
  put_u32(s, (uint32_t)v.size());
  s += v;
}

struct Reader {
  const std::string& s;
  size_t pos = 0;
  explicit Reader(const std::string& str) : s(str) {}
  uint32_t u32() {
    if (pos + 4 > s.size()) throw std::runtime_error("store: truncated frame");
    uint32_t v;
    std::memcpy(&v, s.data() + pos, 4);
    pos += 4;
    return v;
  }
  int64_t i64() {
    if (pos + 8 > s.size()) throw std::runtime_error("store: truncated frame");
    int64_t v;
    std::memcpy(&v, s.data() + pos, 8);
    pos += 8;
    return v;
  }
  std::string str() {
    uint32_t n = u32();
    if (pos + n > s.size()) throw std::runtime_error("store: truncated frame");
    std::string v = s.substr(pos, n);
    pos += n;
    return v;
  }
};

bool write_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd pf{fd, POLLOUT, 0};
        ::poll(&pf, 1, 1000);
        continue;
      }
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

bool read_all(int fd, char* p, size_t n) {
  while (n > 0) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= (size_t)r;
  }
  return true;
}

// Frames are small control messages (keys, ranks' signatures, membership lists); a length past this
// is a corrupt or foreign stream: the connection is dropped instead of buffering without bound.
constexpr uint32_t kMaxFrame = 64u << 20;

void set_nodelay(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

}  // namespace

// ------------------------------------------------------------------------------------------ //
// Server
// ------------------------------------------------------------------------------------------ //
struct StoreServer::Conn {
  int fd;
  std::string in;
  bool dead = false;
};

struct StoreServer::Waiter {
  int fd;
  uint8_t op;  // kGet or kWait
  std::vector<std::string> keys;
  bool has_deadline;
  Clock::time_point deadline;
  bool done = false;
};

StoreServer::StoreServer(const std::string& host, int port) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("StoreServer: socket() failed");
  int one = 1;
  ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (host.empty() || host == "0.0.0.0" || host == "*") {
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
  } else if (::inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) {
    ::close(listen_fd_);
    throw std::runtime_error("StoreServer: bad listen address " + host);
  }
  if (::bind(listen_fd_, (sockaddr*)&addr, sizeof(addr)) != 0) {
    int e = errno;
    ::close(listen_fd_);
    throw std::runtime_error("StoreServer: bind(" + host + ":" + std::to_string(port) + ") failed: " + std::strerror(e));
  }
  if (::listen(listen_fd_, 1024) != 0) {
    ::close(listen_fd_);
    throw std::runtime_error("StoreServer: listen() failed");
  }
  socklen_t len = sizeof(addr);
  ::getsockname(listen_fd_, (sockaddr*)&addr, &len);
  port_ = ntohs(addr.sin_port);
  ::fcntl(listen_fd_, F_SETFL, ::fcntl(listen_fd_, F_GETFL) | O_NONBLOCK);
  if (::pipe(wake_fd_) != 0) throw std::runtime_error("StoreServer: pipe() failed");
  thread_ = std::thread([this] { loop(); });
}

StoreServer::~StoreServer() { stop(); }

void StoreServer::stop() {
  if (stop_.exchange(true)) return;
  char c = 1;
  (void)!::write(wake_fd_[1], &c, 1);
  if (thread_.joinable()) thread_.join();
  for (auto& c2 : conns_) ::close(c2->fd);
  conns_.clear();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  ::close(wake_fd_[0]);
  ::close(wake_fd_[1]);
  listen_fd_ = -1;
}

int64_t StoreServer::num_keys() const {
  std::lock_guard<std::mutex> g(mu_);
  return (int64_t)kv_.size();
}

void StoreServer::reply(Conn& c, uint8_t status, const std::string& payload) {
  std::string out;
  put_u32(out, (uint32_t)(payload.size() + 1));
  out.push_back((char)status);
  out += payload;
  if (!write_all(c.fd, out.data(), out.size())) c.dead = true;
}

bool StoreServer::ready_for(const Waiter& w) const {
  for (const auto& k : w.keys)
    if (kv_.find(k) == kv_.end()) return false;
  return true;
}

void StoreServer::answer(Waiter& w, bool timed_out) {
  Conn* c = nullptr;
  for (auto& cc : conns_)
    if (cc->fd == w.fd) c = cc.get();
  w.done = true;
  if (c == nullptr || c->dead) return;
  if (timed_out) {
    reply(*c, kTimeout, "");
  } else if (w.op == kGet) {
    reply(*c, kOk, kv_.at(w.keys[0]));
  } else {
    reply(*c, kOk, "");
  }
}

void StoreServer::wake_waiters() {
  for (auto& w : waiters_)
    if (!w.done && ready_for(w)) answer(w, false);
  waiters_.erase(std::remove_if(waiters_.begin(), waiters_.end(), [](const Waiter& w) { return w.done; }),
                 waiters_.end());
}

void StoreServer::handle(Conn& c, uint8_t op, const std::string& payload) {
  Reader r(payload);
  std::lock_guard<std::mutex> g(mu_);
  switch (op) {
    case kSet: {
      std::string k = r.str();
      kv_[k] = r.str();
      reply(c, kOk, "");
      wake_waiters();
      break;
    }
    case kAppend: {
      std::string k = r.str();
      kv_[k] += r.str();
      reply(c, kOk, "");
      wake_waiters();
      break;
    }
    case kGet:
    case kWait: {
      Waiter w;
      w.fd = c.fd;
      w.op = op;
      if (op == kGet) {
        w.keys.push_back(r.str());
      } else {
        uint32_t n = r.u32();
        for (uint32_t i = 0; i < n; ++i) w.keys.push_back(r.str());
      }
      int64_t ms = r.i64();
      w.has_deadline = ms >= 0;
      w.deadline = Clock::now() + std::chrono::milliseconds(std::max<int64_t>(ms, 0));
      if (ready_for(w)) {
        answer(w, false);
      } else if (w.has_deadline && ms == 0) {
        answer(w, true);
      } else {
        waiters_.push_back(std::move(w));
      }
      break;
    }
    case kAdd: {
      std::string k = r.str();
      int64_t d = r.i64();
      int64_t v = 0;
      auto it = kv_.find(k);
      if (it != kv_.end() && !it->second.empty()) v = std::stoll(it->second);
      v += d;
      kv_[k] = std::to_string(v);
      std::string out;
      put_i64(out, v);
      reply(c, kOk, out);
      wake_waiters();
      break;
    }
    case kCheck: {
      uint32_t n = r.u32();
      bool all = true;
      for (uint32_t i = 0; i < n; ++i)
        if (kv_.find(r.str()) == kv_.end()) all = false;
      reply(c, kOk, std::string(1, all ? '\1' : '\0'));
      break;
    }
    case kCompareSet: {
      std::string k = r.str(), expected = r.str(), desired = r.str();
      auto it = kv_.find(k);
      if ((it == kv_.end() && expected.empty()) || (it != kv_.end() && it->second == expected)) {
        kv_[k] = desired;
        reply(c, kOk, desired);
        wake_waiters();
      } else {
        reply(c, kOk, it == kv_.end() ? expected : it->second);
      }
      break;
    }
    case kDelete: {
      bool had = kv_.erase(r.str()) > 0;
      reply(c, kOk, std::string(1, had ? '\1' : '\0'));
      break;
    }
    case kNumKeys: {
      std::string out;
      put_i64(out, (int64_t)kv_.size());
      reply(c, kOk, out);
      break;
    }
    case kPing:
      reply(c, kOk, "");
      break;
    default:
      reply(c, kError, "unknown op");
  }
}

void StoreServer::loop() {
  std::vector<pollfd> pfds;
  char buf[65536];
  while (!stop_.load()) {
    pfds.clear();
    pfds.push_back({listen_fd_, POLLIN, 0});
    pfds.push_back({wake_fd_[0], POLLIN, 0});
    for (auto& c : conns_) pfds.push_back({c->fd, POLLIN, 0});
    int timeout_ms = 200;
    {
      auto now = Clock::now();
      for (const auto& w : waiters_)
        if (w.has_deadline) {
          auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(w.deadline - now).count();
          timeout_ms = (int)std::max<int64_t>(0, std::min<int64_t>(timeout_ms, ms + 1));
        }
    }
    int n = ::poll(pfds.data(), pfds.size(), timeout_ms);
    if (n < 0 && errno != EINTR) break;
    if (stop_.load()) break;
    if (n > 0) {
      if (pfds[0].revents & POLLIN) {
        for (;;) {
          int fd = ::accept(listen_fd_, nullptr, nullptr);
          if (fd < 0) break;
          set_nodelay(fd);
          auto c = std::make_unique<Conn>();
          c->fd = fd;
          conns_.push_back(std::move(c));
          nconn_.fetch_add(1);
        }
      }
      for (size_t i = 2; i < pfds.size(); ++i) {
        if (!(pfds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
        Conn* c = nullptr;
        for (auto& cc : conns_)
          if (cc->fd == pfds[i].fd) c = cc.get();
        if (c == nullptr) continue;
        ssize_t r = ::recv(c->fd, buf, sizeof(buf), 0);
        if (r <= 0) {
          if (r < 0 && (errno == EINTR || errno == EAGAIN)) continue;
          c->dead = true;
          continue;
        }
        c->in.append(buf, (size_t)r);
        // complete frames
        size_t pos = 0;
        while (c->in.size() - pos >= 5) {
          uint32_t len;
          std::memcpy(&len, c->in.data() + pos, 4);
          if (len < 1 || len > kMaxFrame) {
            c->dead = true;
            pos = c->in.size();
            break;
          }
          if (c->in.size() - pos - 4 < len) break;
          uint8_t op = (uint8_t)c->in[pos + 4];
          std::string payload = c->in.substr(pos + 5, len - 1);
          pos += 4 + len;
          try {
            handle(*c, op, payload);
          } catch (const std::exception& e) {
            reply(*c, kError, e.what());
          }
        }
        c->in.erase(0, pos);
      }
    }
    // expire waiters, drop dead connections (and their waiters)
    {
      std::lock_guard<std::mutex> g(mu_);
      auto now = Clock::now();
      for (auto& w : waiters_)
        if (!w.done && w.has_deadline && now >= w.deadline) answer(w, true);
      for (auto& c : conns_)
        if (c->dead)
          for (auto& w : waiters_)
            if (w.fd == c->fd) w.done = true;
      waiters_.erase(std::remove_if(waiters_.begin(), waiters_.end(), [](const Waiter& w) { return w.done; }),
                     waiters_.end());
    }
    for (auto& c : conns_)
      if (c->dead) {
        ::close(c->fd);
        nconn_.fetch_sub(1);
      }
    conns_.erase(std::remove_if(conns_.begin(), conns_.end(), [](const std::unique_ptr<Conn>& c) { return c->dead; }),
                 conns_.end());
  }
}

// ------------------------------------------------------------------------------------------ //
// Client
// ------------------------------------------------------------------------------------------ //
StoreClient::StoreClient(const std::string& host, int port, double connect_timeout_s) : host_(host), port_(port) {
  auto deadline = Clock::now() + std::chrono::milliseconds((int64_t)(connect_timeout_s * 1000));
  std::string err;
  for (;;) {
    addrinfo hints{};
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    int rc = ::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
    if (rc == 0 && res != nullptr) {
      int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        ::freeaddrinfo(res);
        fd_ = fd;
        set_nodelay(fd_);
        return;
      }
      err = std::strerror(errno);
      if (fd >= 0) ::close(fd);
      ::freeaddrinfo(res);
    } else {
      err = ::gai_strerror(rc);
    }
    if (Clock::now() >= deadline)
      throw std::runtime_error("StoreClient: cannot connect to " + host + ":" + std::to_string(port) + ": " + err);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

StoreClient::~StoreClient() { close(); }

void StoreClient::close() {
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

uint8_t StoreClient::request(uint8_t op, const std::string& payload, std::string* out) {
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ < 0) throw std::runtime_error("StoreClient: closed");
  std::string frame;
  put_u32(frame, (uint32_t)(payload.size() + 1));
  frame.push_back((char)op);
  frame += payload;
  if (!write_all(fd_, frame.data(), frame.size())) throw std::runtime_error("StoreClient: connection lost (send)");
  uint32_t len;
  if (!read_all(fd_, (char*)&len, 4) || len < 1) throw std::runtime_error("StoreClient: connection lost (recv)");
  if (len > kMaxFrame) throw std::runtime_error("StoreClient: corrupt reply frame");
  std::string body(len, '\0');
  if (!read_all(fd_, &body[0], len)) throw std::runtime_error("StoreClient: connection lost (recv)");
  uint8_t status = (uint8_t)body[0];
  if (status == kError) throw std::runtime_error("StoreClient: server error: " + body.substr(1));
  if (out) *out = body.substr(1);
  return status;
}

static int64_t to_ms(double s) { return s < 0 ? -1 : (int64_t)(s * 1000.0 + 0.5); }

void StoreClient::set(const std::string& key, const std::string& value) {
  std::string p;
  put_str(p, key);
  put_str(p, value);
  request(kSet, p, nullptr);
}

void StoreClient::append(const std::string& key, const std::string& value) {
  std::string p;
  put_str(p, key);
  put_str(p, value);
  request(kAppend, p, nullptr);
}

bool StoreClient::try_get(const std::string& key, double timeout_s, std::string* value) {
  std::string p;
  put_str(p, key);
  put_i64(p, to_ms(timeout_s));
  return request(kGet, p, value) == kOk;
}

std::string StoreClient::get(const std::string& key, double timeout_s) {
  std::string v;
  if (!try_get(key, timeout_s, &v)) throw std::runtime_error("StoreClient: timeout waiting for key '" + key + "'");
  return v;
}

int64_t StoreClient::add(const std::string& key, int64_t delta) {
  std::string p, out;
  put_str(p, key);
  put_i64(p, delta);
  request(kAdd, p, &out);
  Reader r(out);
  return r.i64();
}

bool StoreClient::check(const std::vector<std::string>& keys) {
  std::string p, out;
  put_u32(p, (uint32_t)keys.size());
  for (const auto& k : keys) put_str(p, k);
  request(kCheck, p, &out);
  return !out.empty() && out[0] == '\1';
}

bool StoreClient::wait(const std::vector<std::string>& keys, double timeout_s) {
  std::string p;
  put_u32(p, (uint32_t)keys.size());
  for (const auto& k : keys) put_str(p, k);
  put_i64(p, to_ms(timeout_s));
  return request(kWait, p, nullptr) == kOk;
}

std::string StoreClient::compare_set(const std::string& key, const std::string& expected, const std::string& desired) {
  std::string p, out;
  put_str(p, key);
  put_str(p, expected);
  put_str(p, desired);
  request(kCompareSet, p, &out);
  return out;
}

bool StoreClient::del(const std::string& key) {
  std::string p, out;
  put_str(p, key);
  request(kDelete, p, &out);
  return !out.empty() && out[0] == '\1';
}

int64_t StoreClient::num_keys() {
  std::string out;
  request(kNumKeys, "", &out);
  Reader r(out);
  return r.i64();
}

}  // namespace mihvd

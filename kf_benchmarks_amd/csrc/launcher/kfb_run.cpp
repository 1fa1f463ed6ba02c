// kfb-run: single-node multi-process launcher (the role of KungFu's Go
// `kungfu-run -np N prog args...`, tcb/README.md:95-105, tcb/run_kf.sh).
//
// Spawns N peers of one command, one per GPU, with the torch.distributed
// rendezvous variables (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
// MASTER_ADDR / MASTER_PORT) plus KungFu-style peer specs
// (KUNGFU_SELF_SPEC=127.0.0.1:<port>, KUNGFU_INIT_PEERS).  Each peer's stdout
// and stderr are
//   * echoed line by line with a coloured "[127.0.0.1.<port>::stdout] " prefix
//     (stderr tagged in magenta), as kungfu-run does, and
//   * written to <logdir>/127.0.0.1.<port>.{stdout,stderr}.log.
// Fail-fast: the first peer that exits non-zero (or dies on a signal) makes
// the launcher terminate the remaining peers (SIGTERM to their process
// groups, SIGKILL after a grace period) and exit 1 with
// "exit on error: <k> tasks failed".
//
// usage: kfb-run -np N [-port-range 10000-11000] [-logdir DIR] [-q]
//                [-timeout SECONDS] [-H 127.0.0.1:N] [-master-port P] [-chief-only]
//                prog args...
// -chief-only echoes rank 0's output unprefixed and keeps the other ranks'
// output in their log files only (used when one --num_gpus=N command is run
// as N tower processes, so the console looks like a single-process run).

#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <netinet/in.h>
#include <arpa/inet.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct Stream {
  int fd = -1;
  FILE* log = nullptr;
  std::string pending;
  bool is_err = false;
};

struct Peer {
  int rank = 0;
  int port = 0;
  pid_t pid = -1;
  bool running = false;
  int status = 0;
  Stream out, err;
  std::string name() const { return "127.0.0.1." + std::to_string(port); }
};

const char* kColors[] = {"\x1b[1;32m", "\x1b[1;34m", "\x1b[1;33m", "\x1b[1;36m",
                         "\x1b[1;31m", "\x1b[1;37m", "\x1b[0;32m", "\x1b[0;34m"};
const char* kReset = "\x1b[m";
const char* kMagenta = "\x1b[1;35m";

volatile sig_atomic_t g_signal = 0;
void on_signal(int s) { g_signal = s; }

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

void usage() {
  fprintf(stderr,
          "usage: kfb-run -np N [-port-range LO-HI] [-logdir DIR] [-q] [-timeout S]\n"
          "               [-H 127.0.0.1:N] [-master-port P] prog [args...]\n");
}

bool port_free(int port) {
  int s = socket(AF_INET, SOCK_STREAM, 0);
  if (s < 0) return false;
  int one = 1;
  setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = inet_addr("127.0.0.1");
  bool ok = bind(s, (sockaddr*)&a, sizeof(a)) == 0;
  close(s);
  return ok;
}

// An ephemeral port from the kernel (bind to port 0): concurrent launches
// on one host never pick the same rendezvous port, unlike a scan upward
// from the peer ports.
int ephemeral_port() {
  int s = socket(AF_INET, SOCK_STREAM, 0);
  if (s < 0) return -1;
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = 0;
  a.sin_addr.s_addr = inet_addr("127.0.0.1");
  int port = -1;
  socklen_t len = sizeof(a);
  if (bind(s, (sockaddr*)&a, sizeof(a)) == 0 && getsockname(s, (sockaddr*)&a, &len) == 0)
    port = ntohs(a.sin_port);
  close(s);
  return port;
}

bool g_chief_only = false;  // -chief-only: echo rank 0 verbatim, others to logs only

void emit(Peer& p, Stream& s, const std::string& line, bool quiet, int color) {
  if (s.log) {
    fwrite(line.data(), 1, line.size(), s.log);
    fputc('\n', s.log);
    fflush(s.log);
  }
  if (g_chief_only) {
    if (p.rank != 0) return;
    FILE* o = s.is_err ? stderr : stdout;
    fprintf(o, "%s\n", line.c_str());
    fflush(o);
    return;
  }
  if (quiet) return;
  FILE* o = s.is_err ? stderr : stdout;
  if (s.is_err)
    fprintf(o, "[%s%s%s::%sstderr%s] %s\n", kColors[color % 8], p.name().c_str(), kReset,
            kMagenta, kReset, line.c_str());
  else
    fprintf(o, "[%s%s%s::stdout] %s\n", kColors[color % 8], p.name().c_str(), kReset,
            line.c_str());
  fflush(o);
}

// Returns false on EOF.
bool pump(Peer& p, Stream& s, bool quiet, int color) {
  char buf[65536];
  ssize_t n = read(s.fd, buf, sizeof(buf));
  if (n < 0 && (errno == EINTR || errno == EAGAIN)) return true;
  if (n <= 0) {
    if (!s.pending.empty()) emit(p, s, s.pending, quiet, color);
    s.pending.clear();
    close(s.fd);
    s.fd = -1;
    return false;
  }
  s.pending.append(buf, (size_t)n);
  size_t start = 0, nl;
  while ((nl = s.pending.find('\n', start)) != std::string::npos) {
    emit(p, s, s.pending.substr(start, nl - start), quiet, color);
    start = nl + 1;
  }
  s.pending.erase(0, start);
  return true;
}

void kill_all(std::vector<Peer>& peers, int sig) {
  for (auto& p : peers)
    if (p.running) kill(-p.pid, sig);
}

}  // namespace

int main(int argc, char** argv) {
  int np = -1, port_lo = 10000, port_hi = 11000, master_port = -1;
  double timeout = 0.0, grace = 10.0;
  bool quiet = false;
  std::string logdir = ".";
  int i = 1;
  for (; i < argc; ++i) {
    std::string a = argv[i];
    auto need = [&](const char* what) -> const char* {
      if (i + 1 >= argc) {
        fprintf(stderr, "kfb-run: %s needs a value\n", what);
        exit(2);
      }
      return argv[++i];
    };
    if (a == "-np") {
      np = atoi(need("-np"));
    } else if (a == "-port-range") {
      std::string r = need("-port-range");
      if (sscanf(r.c_str(), "%d-%d", &port_lo, &port_hi) != 2 || port_hi <= port_lo) {
        fprintf(stderr, "kfb-run: bad -port-range %s\n", r.c_str());
        return 2;
      }
    } else if (a == "-logdir") {
      logdir = need("-logdir");
    } else if (a == "-q") {
      quiet = true;
    } else if (a == "-chief-only") {
      g_chief_only = true;
    } else if (a == "-timeout") {
      timeout = atof(need("-timeout"));
    } else if (a == "-grace") {
      grace = atof(need("-grace"));
    } else if (a == "-master-port") {
      master_port = atoi(need("-master-port"));
    } else if (a == "-H") {
      std::string h = need("-H");
      size_t c = h.rfind(':');
      if (h.substr(0, c) != "127.0.0.1" && h.substr(0, c) != "localhost") {
        fprintf(stderr, "kfb-run: only single-node runs (-H 127.0.0.1:N) are supported\n");
        return 2;
      }
      if (np < 0 && c != std::string::npos) np = atoi(h.c_str() + c + 1);
    } else if (a == "-w" || a == "-elastic") {
      fprintf(stderr, "kfb-run: elastic mode is not supported\n");
      return 2;
    } else if (a == "--") {
      ++i;
      break;
    } else if (!a.empty() && a[0] == '-') {
      fprintf(stderr, "kfb-run: unknown option %s\n", a.c_str());
      usage();
      return 2;
    } else {
      break;
    }
  }
  if (np <= 0 || i >= argc) {
    usage();
    return 2;
  }
  // mkdir -p logdir
  for (size_t k = 1; k <= logdir.size(); ++k)
    if (k == logdir.size() || logdir[k] == '/') mkdir(logdir.substr(0, k).c_str(), 0755);
  std::vector<char*> cmd(argv + i, argv + argc);
  cmd.push_back(nullptr);

  // peer ports: np consecutive free ports from port_lo (KungFu: 10000 + i)
  std::vector<int> ports;
  for (int p = port_lo; p < port_hi && (int)ports.size() < np; ++p)
    if (port_free(p)) ports.push_back(p);
  if ((int)ports.size() < np) {
    fprintf(stderr, "kfb-run: not enough free ports in %d-%d\n", port_lo, port_hi);
    return 2;
  }
  if (master_port < 0) master_port = ephemeral_port();
  if (master_port < 0) {
    for (int p = ports.back() + 1; p < 65535; ++p)
      if (port_free(p)) {
        master_port = p;
        break;
      }
  }
  std::string peers_spec;
  for (int r = 0; r < np; ++r)
    peers_spec += (r ? "," : "") + std::string("127.0.0.1:") + std::to_string(ports[r]);

  if (!quiet && !g_chief_only) {
    fprintf(stdout, "[I] will parallel run %d instances of %s with [", np, cmd[0]);
    for (size_t k = 1; cmd[k]; ++k) fprintf(stdout, "%s\"%s\"", k > 1 ? " " : "", cmd[k]);
    fprintf(stdout, "]\n");
    fflush(stdout);
  }

  signal(SIGINT, on_signal);
  signal(SIGTERM, on_signal);
  signal(SIGPIPE, SIG_IGN);

  std::vector<Peer> peers(np);
  double t0 = now_s();
  for (int r = 0; r < np; ++r) {
    Peer& p = peers[r];
    p.rank = r;
    p.port = ports[r];
    int po[2], pe[2];
    if (pipe(po) || pipe(pe)) {
      perror("pipe");
      kill_all(peers, SIGKILL);
      return 1;
    }
    std::string base = logdir + "/" + p.name();
    p.out.log = fopen((base + ".stdout.log").c_str(), "w");
    p.err.log = fopen((base + ".stderr.log").c_str(), "w");
    p.err.is_err = true;
    if (!p.out.log || !p.err.log)
      fprintf(stderr, "kfb-run: cannot write logs under %s: %s\n", logdir.c_str(), strerror(errno));
    pid_t pid = fork();
    if (pid < 0) {
      perror("fork");
      kill_all(peers, SIGKILL);
      return 1;
    }
    if (pid == 0) {
      setpgid(0, 0);
      dup2(po[1], 1);
      dup2(pe[1], 2);
      close(po[0]);
      close(po[1]);
      close(pe[0]);
      close(pe[1]);
      setenv("RANK", std::to_string(r).c_str(), 1);
      setenv("LOCAL_RANK", std::to_string(r).c_str(), 1);
      setenv("WORLD_SIZE", std::to_string(np).c_str(), 1);
      setenv("LOCAL_WORLD_SIZE", std::to_string(np).c_str(), 1);
      setenv("GROUP_RANK", "0", 1);
      setenv("MASTER_ADDR", "127.0.0.1", 1);
      setenv("MASTER_PORT", std::to_string(master_port).c_str(), 1);
      setenv("KUNGFU_SELF_SPEC", ("127.0.0.1:" + std::to_string(p.port)).c_str(), 1);
      setenv("KUNGFU_INIT_PEERS", peers_spec.c_str(), 1);
      setenv("KFB_LAUNCHER", "kfb-run", 1);
      setenv("PYTHONUNBUFFERED", "1", 0);
      setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 0);
      execvp(cmd[0], cmd.data());
      fprintf(stderr, "kfb-run: cannot exec %s: %s\n", cmd[0], strerror(errno));
      _exit(127);
    }
    setpgid(pid, pid);
    close(po[1]);
    close(pe[1]);
    p.pid = pid;
    p.running = true;
    p.out.fd = po[0];
    p.err.fd = pe[0];
  }

  int failed = 0, finished = 0;
  bool stopping = false;
  double stop_at = 0.0;
  for (;;) {
    std::vector<pollfd> fds;
    std::vector<std::pair<int, Stream*>> who;
    for (int r = 0; r < np; ++r)
      for (Stream* s : {&peers[r].out, &peers[r].err})
        if (s->fd >= 0) {
          fds.push_back({s->fd, POLLIN, 0});
          who.push_back({r, s});
        }
    if (!fds.empty()) {
      int rc = poll(fds.data(), fds.size(), 200);
      if (rc > 0)
        for (size_t k = 0; k < fds.size(); ++k)
          if (fds[k].revents & (POLLIN | POLLHUP | POLLERR))
            pump(peers[who[k].first], *who[k].second, quiet, who[k].first);
    } else {
      usleep(50 * 1000);
    }
    // reap
    for (auto& p : peers) {
      if (!p.running) continue;
      int st;
      pid_t w = waitpid(p.pid, &st, WNOHANG);
      if (w != p.pid) continue;
      p.running = false;
      p.status = st;
      ++finished;
      bool ok = WIFEXITED(st) && WEXITSTATUS(st) == 0;
      if (!ok) {
        ++failed;
        if (WIFEXITED(st))
          fprintf(stderr, "%s[E]%s #<%s> exited with error: exit status %d\n", kMagenta, kReset,
                  p.name().c_str(), WEXITSTATUS(st));
        else
          fprintf(stderr, "%s[E]%s #<%s> exited with error: signal %d\n", kMagenta, kReset,
                  p.name().c_str(), WTERMSIG(st));
        if (!stopping) {  // fail fast
          stopping = true;
          stop_at = now_s();
          kill_all(peers, SIGTERM);
        }
      }
    }
    if (g_signal && !stopping) {
      stopping = true;
      stop_at = now_s();
      kill_all(peers, SIGTERM);
    }
    if (timeout > 0 && !stopping && now_s() - t0 > timeout) {
      fprintf(stderr, "[E] timeout after %.0fs, stopping all peers\n", timeout);
      stopping = true;
      stop_at = now_s();
      ++failed;
      kill_all(peers, SIGTERM);
    }
    if (stopping && now_s() - stop_at > grace) kill_all(peers, SIGKILL);
    bool streams_open = false;
    for (auto& p : peers) streams_open |= p.out.fd >= 0 || p.err.fd >= 0;
    if (finished == np && !streams_open) break;
    if (finished == np && stopping && now_s() - stop_at > grace) break;
  }
  for (auto& p : peers) {
    if (p.out.log) fclose(p.out.log);
    if (p.err.log) fclose(p.err.log);
  }
  if (!g_chief_only) {
    fprintf(stdout, "[I] all %d/%d local peers finished, took %.3fs\n", finished, np,
            now_s() - t0);
    fflush(stdout);
  }
  if (failed) {
    fprintf(stderr, "exit on error: %d tasks failed\n", failed);
    return 1;
  }
  return g_signal ? 128 + g_signal : 0;
}

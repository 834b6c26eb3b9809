// anxrun — start N ranks of a program on this node (the reference's `mpirun --oversubscribe -np N
// ./template`, scripts/common_test_utils.sh:271-279).
//
//   anxrun -np N [--timeout SEC] [--port P] [--] program [args...]
//
// Each rank gets ANX_RANK / ANX_LOCAL_RANK / ANX_WORLD_SIZE / ANX_LOCAL_WORLD_SIZE / ANX_NNODES /
// ANX_MASTER_ADDR / ANX_MASTER_PORT
// (rendezvous on 127.0.0.1). Ranks bind GPU `local_rank % device_count` themselves — the binding
// the reference documents but never calls. Fail-stop like MPI_Abort: the first rank
// that exits nonzero (or dies on a signal) takes the job down; a watchdog timeout exits 124.
// The launcher itself never touches the GPU, so exec'ing the ranks is safe.
#include <netinet/in.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static int free_port() {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof a);
  socklen_t len = sizeof a;
  getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
  const int p = ntohs(a.sin_port);
  close(fd);
  return p;
}

static void usage() {
  std::fprintf(stderr, "usage: anxrun -np N [--timeout SEC] [--port P] [--] program [args...]\n");
  std::exit(2);
}

int main(int argc, char** argv) {
  // Multi-node (the reference's hostfile runs, scripts/2_final_multi_machine.sh:396-410): start
  // `anxrun -np <per node> --nnodes K --node-rank R --master-addr <node 0> --port P` on every node;
  // global rank = R * np + local rank.
  int np = 1, port = 0, nnodes = 1, node_rank = 0;
  std::string master = "127.0.0.1";
  double timeout = 0;
  int i = 1;
  for (; i < argc; ++i) {
    std::string a = argv[i];
    if ((a == "-np" || a == "-n" || a == "--np") && i + 1 < argc) {
      np = std::atoi(argv[++i]);
    } else if (a == "--timeout" && i + 1 < argc) {
      timeout = std::atof(argv[++i]);
    } else if (a == "--port" && i + 1 < argc) {
      port = std::atoi(argv[++i]);
    } else if (a == "--nnodes" && i + 1 < argc) {
      nnodes = std::atoi(argv[++i]);
    } else if (a == "--node-rank" && i + 1 < argc) {
      node_rank = std::atoi(argv[++i]);
    } else if (a == "--master-addr" && i + 1 < argc) {
      master = argv[++i];
    } else if (a == "--") {
      ++i;
      break;
    } else {
      break;
    }
  }
  if (i >= argc || np < 1 || nnodes < 1 || node_rank < 0 || node_rank >= nnodes) usage();
  if (!port) {
    if (nnodes > 1) {
      std::fprintf(stderr, "anxrun: --port is required with --nnodes > 1\n");
      return 2;
    }
    port = free_port();
  }
  std::vector<pid_t> kids;
  for (int r = 0; r < np; ++r) {
    pid_t pid = fork();
    if (pid < 0) {
      std::perror("fork");
      return 1;
    }
    if (pid == 0) {
      setenv("ANX_RANK", std::to_string(node_rank * np + r).c_str(), 1);
      setenv("ANX_LOCAL_RANK", std::to_string(r).c_str(), 1);
      setenv("ANX_WORLD_SIZE", std::to_string(np * nnodes).c_str(), 1);
      setenv("ANX_LOCAL_WORLD_SIZE", std::to_string(np).c_str(), 1);  // ranks on this node
      setenv("ANX_NNODES", std::to_string(nnodes).c_str(), 1);
      setenv("ANX_MASTER_ADDR", master.c_str(), 1);
      setenv("ANX_MASTER_PORT", std::to_string(port).c_str(), 1);
      execvp(argv[i], argv + i);
      std::perror("execvp");
      std::_Exit(127);
    }
    kids.push_back(pid);
  }
  const auto t0 = std::chrono::steady_clock::now();
  int rc = 0, alive = np;
  auto kill_all = [&](int sig) {
    for (pid_t k : kids)
      if (k > 0) kill(k, sig);
  };
  while (alive > 0) {
    int status = 0;
    pid_t p = waitpid(-1, &status, WNOHANG);
    if (p > 0) {
      for (pid_t& k : kids)
        if (k == p) k = -1;
      --alive;
      int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
      if (code != 0 && rc == 0) {
        rc = code;
        std::fprintf(stderr, "anxrun: a rank exited with %d; stopping the job\n", code);
        kill_all(SIGTERM);
      }
      continue;
    }
    if (timeout > 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout) {
      std::fprintf(stderr, "anxrun: watchdog timeout after %.0f s\n", timeout);
      kill_all(SIGKILL);
      rc = 124;
      timeout = 0;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  return rc;
}

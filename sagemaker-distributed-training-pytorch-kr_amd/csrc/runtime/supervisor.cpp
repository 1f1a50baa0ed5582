// Native rank supervisor: fork one process per GPU, fail fast, clean up the whole group.
//
// Replaces the reference's `mpirun ... -mca orte_abort_on_non_zero_status 1` launcher (SURVEY
// C5/E4, NB1:686) and SageMaker's `max_run` wall-clock limit (NB1:361-366): every rank runs in
// one process group; the first rank that exits non-zero (or dies on a signal) makes the
// supervisor SIGTERM the group, wait `grace` seconds, then SIGKILL what is left; its status
// becomes the job status. `max_run` seconds with no completion kills the group (status 124).
//
// The children exec immediately after fork, before anything touches a GPU, and the supervisor
// itself never initialises one (safe with the HIP runtime).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <csignal>
#include <cstring>
#include <ctime>
#include <string>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

namespace py = pybind11;

namespace {

volatile sig_atomic_t g_forward_signal = 0;

void on_signal(int sig) { g_forward_signal = sig; }

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int decode_status(int st) {
  if (WIFEXITED(st)) return WEXITSTATUS(st);
  if (WIFSIGNALED(st)) return 128 + WTERMSIG(st);
  return 1;
}

// Returns (job_status, per-rank statuses, first_failed_rank or -1).
py::tuple run_ranks(const std::vector<std::vector<std::string>>& argvs,
                    const std::vector<std::vector<std::string>>& envs, double grace, double max_run,
                    const std::string& cwd, int out_fd) {
  const size_t n = argvs.size();
  if (n == 0 || envs.size() != n) throw std::invalid_argument("run_ranks: need one argv and one env per rank");
  std::vector<pid_t> pids(n, -1);
  std::vector<int> status(n, -1);
  pid_t pgid = 0;
  struct sigaction sa, old_int, old_term;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_signal;
  sigaction(SIGINT, &sa, &old_int);
  sigaction(SIGTERM, &sa, &old_term);
  g_forward_signal = 0;

  for (size_t r = 0; r < n; ++r) {
    // Build argv / envp before fork (no allocation in the child).
    std::vector<char*> av, ev;
    for (auto& s : argvs[r]) av.push_back(const_cast<char*>(s.c_str()));
    av.push_back(nullptr);
    for (auto& s : envs[r]) ev.push_back(const_cast<char*>(s.c_str()));
    ev.push_back(nullptr);
    pid_t pid = fork();
    if (pid < 0) throw std::runtime_error("fork failed");
    if (pid == 0) {
      setpgid(0, pgid);  // first child creates the group, the rest join it
      signal(SIGINT, SIG_DFL);
      signal(SIGTERM, SIG_DFL);
      if (!cwd.empty() && chdir(cwd.c_str()) != 0) _exit(126);
      if (out_fd >= 0) {  // merge the rank's stdout/stderr into the supervisor's log pipe
        dup2(out_fd, 1);
        dup2(out_fd, 2);
        if (out_fd > 2) close(out_fd);
      }
      execvpe(av[0], av.data(), ev.data());
      _exit(127);
    }
    if (pgid == 0) pgid = pid;
    setpgid(pid, pgid);
    pids[r] = pid;
  }

  int job = 0, first_failed = -1;
  size_t alive = n;
  bool killing = false;
  double kill_at = 0.0;
  const double t0 = now_s();
  {
    py::gil_scoped_release nogil;
    while (alive > 0) {
      int st = 0;
      pid_t p = waitpid(-pgid, &st, WNOHANG);
      if (p > 0) {
        for (size_t r = 0; r < n; ++r) {
          if (pids[r] == p) {
            status[r] = decode_status(st);
            --alive;
            if (status[r] != 0 && first_failed < 0 && !killing) {
              first_failed = (int)r;
              job = status[r];
            }
          }
        }
        continue;
      }
      if (p < 0 && errno == ECHILD) break;
      const double t = now_s();
      if (!killing) {
        bool fail = first_failed >= 0 || g_forward_signal != 0;
        if (max_run > 0 && t - t0 > max_run) {
          fail = true;
          if (job == 0) job = 124;
        }
        if (g_forward_signal && job == 0) job = 128 + g_forward_signal;
        if (fail && alive > 0) {
          kill(-pgid, SIGTERM);
          killing = true;
          kill_at = t + grace;
        }
      } else if (t > kill_at) {
        kill(-pgid, SIGKILL);
        kill_at = t + 3600.0;
      }
      usleep(20000);
    }
  }
  sigaction(SIGINT, &old_int, nullptr);
  sigaction(SIGTERM, &old_term, nullptr);
  return py::make_tuple(job, status, first_failed);
}

}  // namespace

void register_supervisor(py::module_& m) {
  m.def("run_ranks", &run_ranks, py::arg("argvs"), py::arg("envs"), py::arg("grace") = 10.0,
        py::arg("max_run") = 0.0, py::arg("cwd") = std::string(), py::arg("out_fd") = -1,
        "Fork/exec one process per rank in a shared process group; fail fast on the first "
        "non-zero exit; returns (job_status, [rank statuses], first_failed_rank).");
}

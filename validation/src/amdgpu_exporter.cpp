// amdgpu-exporter: a small native Prometheus exporter for MI355X nodes, built
// on the AMD SMI library (libamd_smi). It is the "rocm-smi exporter DaemonSet"
// of BASELINE config #4, and the GPU-metrics source for the CNPack Prometheus
// examples when modules/amd-gpu-stack runs in daemonsets mode. It replaces
// the reference's implicit DCGM exporter (bundled in the NVIDIA GPU Operator
// chart installed at /root/reference/eks/main.tf:185-203).
//
// Modes:
//   amdgpu-exporter [--port 9400]          serve GET /metrics and /healthz
//   amdgpu-exporter --once                 print one scrape to stdout and exit
//   amdgpu-exporter --textfile F [--interval S]
//                                          rewrite F atomically every S seconds
//                                          (node-exporter textfile collector)
//
// One gpu_metrics read per GPU per scrape (a single sysfs blob: activity,
// power, temperatures, clocks, throttle status, xGMI traffic), plus VRAM
// usage and ECC totals. Values the firmware reports as unsupported (all-ones)
// are skipped instead of exported as 65535.
#include <amd_smi/amdsmi.h>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

struct Family {
  std::string help, type;
  std::vector<std::string> samples;  // already formatted "labels value"
};

class Scrape {
 public:
  void add(const std::string& name, const std::string& help, const std::string& type,
           const std::string& labels, double v) {
    auto& f = fam_[name];
    f.help = help;
    f.type = type;
    char b[64];
    std::snprintf(b, sizeof b, "%.10g", v);
    f.samples.push_back((labels.empty() ? "" : "{" + labels + "}") + " " + b);
  }
  std::string text() const {
    std::ostringstream o;
    for (const auto& [name, f] : fam_) {
      o << "# HELP " << name << " " << f.help << "\n# TYPE " << name << " " << f.type << "\n";
      for (const auto& s : f.samples) o << name << s << "\n";
    }
    return o.str();
  }

 private:
  std::map<std::string, Family> fam_;
};

bool ok16(uint16_t v) { return v != 0xFFFF; }
bool ok32(uint32_t v) { return v != 0xFFFFFFFFu; }
bool ok64(uint64_t v) { return v != 0xFFFFFFFFFFFFFFFFull; }
// ECC totals: MI355X firmware reports 2^47 (bit 47 alone) for a counter it
// does not provide (seen on the correctable count); no real count gets there.
bool ok_count(uint64_t v) { return v < (1ull << 47); }

std::string bdf_str(amdsmi_processor_handle h) {
  amdsmi_bdf_t b;
  if (amdsmi_get_gpu_device_bdf(h, &b) != AMDSMI_STATUS_SUCCESS) return "unknown";
  char s[32];
  std::snprintf(s, sizeof s, "%04x:%02x:%02x.%x", (unsigned)b.domain_number,
                (unsigned)b.bus_number, (unsigned)b.device_number, (unsigned)b.function_number);
  return s;
}

std::vector<amdsmi_processor_handle> gpus() {
  std::vector<amdsmi_processor_handle> out;
  uint32_t ns = 0;
  if (amdsmi_get_socket_handles(&ns, nullptr) != AMDSMI_STATUS_SUCCESS || ns == 0) return out;
  std::vector<amdsmi_socket_handle> socks(ns);
  if (amdsmi_get_socket_handles(&ns, socks.data()) != AMDSMI_STATUS_SUCCESS) return out;
  for (auto s : socks) {
    uint32_t np = 0;
    if (amdsmi_get_processor_handles(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
    std::vector<amdsmi_processor_handle> ps(np);
    if (amdsmi_get_processor_handles(s, &np, ps.data()) != AMDSMI_STATUS_SUCCESS) continue;
    out.insert(out.end(), ps.begin(), ps.begin() + np);
  }
  return out;
}

std::string collect(bool smi_up) {
  const auto t0 = std::chrono::steady_clock::now();
  Scrape sc;
  std::vector<amdsmi_processor_handle> hs;
  if (smi_up) hs = gpus();
  sc.add("amdgpu_exporter_up", "1 if the AMD SMI library initialised and found GPUs.", "gauge",
         "", smi_up && !hs.empty() ? 1 : 0);
  sc.add("amdgpu_gpu_count", "GPUs visible to the exporter.", "gauge", "", (double)hs.size());
  for (size_t i = 0; i < hs.size(); ++i) {
    const auto h = hs[i];
    const std::string L = "gpu=\"" + std::to_string(i) + "\",bdf=\"" + bdf_str(h) + "\"";
    amdsmi_gpu_metrics_t m;
    std::memset(&m, 0xFF, sizeof m);
    if (amdsmi_get_gpu_metrics_info(h, &m) == AMDSMI_STATUS_SUCCESS) {
      if (ok16(m.average_gfx_activity))
        sc.add("amdgpu_gfx_activity_percent", "Graphics/compute engine activity.", "gauge", L,
               m.average_gfx_activity);
      if (ok16(m.average_umc_activity))
        sc.add("amdgpu_umc_activity_percent", "HBM memory-controller activity.", "gauge", L,
               m.average_umc_activity);
      double pw = ok16(m.current_socket_power) ? m.current_socket_power
                  : ok16(m.average_socket_power) ? m.average_socket_power : -1;
      if (pw >= 0) sc.add("amdgpu_socket_power_watts", "Socket power.", "gauge", L, pw);
      if (ok16(m.temperature_hotspot))
        sc.add("amdgpu_temperature_celsius", "Temperatures by sensor.", "gauge",
               L + ",sensor=\"hotspot\"", m.temperature_hotspot);
      if (ok16(m.temperature_mem))
        sc.add("amdgpu_temperature_celsius", "Temperatures by sensor.", "gauge",
               L + ",sensor=\"hbm\"", m.temperature_mem);
      double gclk = ok16(m.current_gfxclk) ? m.current_gfxclk
                    : ok16(m.current_gfxclks[0]) ? m.current_gfxclks[0] : -1;
      if (gclk >= 0)
        sc.add("amdgpu_clock_mhz", "Current clocks.", "gauge", L + ",clock=\"gfx\"", gclk);
      if (ok16(m.current_uclk))
        sc.add("amdgpu_clock_mhz", "Current clocks.", "gauge", L + ",clock=\"mem\"", m.current_uclk);
      if (ok32(m.throttle_status))
        sc.add("amdgpu_throttle_status", "Firmware throttle status bits.", "gauge", L,
               m.throttle_status);
      for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
        const std::string LL = L + ",link=\"" + std::to_string(l) + "\"";
        if (ok64(m.xgmi_read_data_acc[l]) && m.xgmi_read_data_acc[l])
          sc.add("amdgpu_xgmi_read_kilobytes_total", "xGMI data read over each link.", "counter",
                 LL, (double)m.xgmi_read_data_acc[l]);
        if (ok64(m.xgmi_write_data_acc[l]) && m.xgmi_write_data_acc[l])
          sc.add("amdgpu_xgmi_write_kilobytes_total", "xGMI data written over each link.",
                 "counter", LL, (double)m.xgmi_write_data_acc[l]);
      }
    }
    uint64_t used = 0, total = 0;
    if (amdsmi_get_gpu_memory_total(h, AMDSMI_MEM_TYPE_VRAM, &total) == AMDSMI_STATUS_SUCCESS)
      sc.add("amdgpu_vram_total_bytes", "HBM capacity.", "gauge", L, (double)total);
    if (amdsmi_get_gpu_memory_usage(h, AMDSMI_MEM_TYPE_VRAM, &used) == AMDSMI_STATUS_SUCCESS)
      sc.add("amdgpu_vram_used_bytes", "HBM in use.", "gauge", L, (double)used);
    amdsmi_error_count_t ec;
    if (amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS) {
      if (ok_count(ec.correctable_count))
        sc.add("amdgpu_ecc_errors_total", "Accumulated ECC errors.", "counter",
               L + ",kind=\"correctable\"", (double)ec.correctable_count);
      if (ok_count(ec.uncorrectable_count))
        sc.add("amdgpu_ecc_errors_total", "Accumulated ECC errors.", "counter",
               L + ",kind=\"uncorrectable\"", (double)ec.uncorrectable_count);
    }
  }
  const double dt =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  sc.add("amdgpu_exporter_scrape_seconds", "Time spent collecting this scrape.", "gauge", "", dt);
  return sc.text();
}

bool write_atomic(const std::string& path, const std::string& body) {
  const std::string tmp = path + ".tmp";
  {
    std::ofstream f(tmp);
    if (!f) return false;
    f << body;
  }
  return std::rename(tmp.c_str(), path.c_str()) == 0;
}

int serve(int port, bool smi_up) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return 2;
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons((uint16_t)port);
  if (bind(fd, (sockaddr*)&a, sizeof a) != 0 || listen(fd, 16) != 0) {
    std::perror("amdgpu-exporter: bind/listen");
    close(fd);
    return 2;
  }
  std::fprintf(stderr, "amdgpu-exporter: serving :%d/metrics\n", port);
  while (!g_stop) {
    const int c = accept(fd, nullptr, nullptr);
    if (c < 0) continue;  // EINTR on SIGTERM -> loop re-checks g_stop
    timeval tv{5, 0};
    setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    char buf[2048];
    const ssize_t n = recv(c, buf, sizeof buf - 1, 0);
    std::string req = n > 0 ? std::string(buf, (size_t)n) : "";
    std::string status = "200 OK", type = "text/plain; version=0.0.4", body;
    if (req.rfind("GET /metrics", 0) == 0) body = collect(smi_up);
    else if (req.rfind("GET /healthz", 0) == 0) body = "ok\n";
    else { status = "404 Not Found"; body = "not found\n"; }
    std::string resp = "HTTP/1.1 " + status + "\r\nContent-Type: " + type +
                       "\r\nContent-Length: " + std::to_string(body.size()) +
                       "\r\nConnection: close\r\n\r\n" + body;
    size_t off = 0;
    while (off < resp.size()) {
      const ssize_t w = send(c, resp.data() + off, resp.size() - off, MSG_NOSIGNAL);
      if (w <= 0) break;
      off += (size_t)w;
    }
    close(c);
  }
  close(fd);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  int port = 9400;
  bool once = false;
  std::string textfile;
  double interval = 15;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
    const char* v = nullptr;
    if (a == "--once") once = true;
    else if (a == "--port" && (v = val())) port = std::atoi(v);
    else if (a == "--textfile" && (v = val())) textfile = v;
    else if (a == "--interval" && (v = val())) interval = std::atof(v);
    else {
      std::fprintf(stderr,
                   "usage: amdgpu-exporter [--port N] | --once | --textfile F [--interval S]\n");
      return 2;
    }
  }
  // no SA_RESTART: a blocked accept() returns EINTR on SIGTERM, so pod
  // termination does not wait for the kubelet's grace period
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = 0;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  const bool smi_up = amdsmi_init(AMDSMI_INIT_AMD_GPUS) == AMDSMI_STATUS_SUCCESS;
  int rc = 0;
  if (once) {
    const std::string t = collect(smi_up);
    std::fwrite(t.data(), 1, t.size(), stdout);
    rc = (smi_up && !gpus().empty()) ? 0 : 2;
  } else if (!textfile.empty()) {
    while (!g_stop) {
      if (!write_atomic(textfile, collect(smi_up))) {
        std::fprintf(stderr, "amdgpu-exporter: cannot write %s\n", textfile.c_str());
        rc = 2;
        break;
      }
      for (double s = 0; s < interval && !g_stop; s += 0.2)
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
    }
  } else {
    rc = serve(port, smi_up);
  }
  if (smi_up) amdsmi_shut_down();
  return rc;
}

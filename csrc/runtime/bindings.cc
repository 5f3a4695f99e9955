// pybind11 bindings of the native runtime: object store, cluster scheduler,
// compiled-graph shm channels, durable GCS table store.
#include <tuple>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "channel.h"
#include "gcs_store.h"
#include "object_store.h"
#include "scheduler.h"

namespace py = pybind11;
using namespace caamd_rt;

// A sealed object's payload exported through the Python buffer protocol. It
// holds a pin on the object for as long as any memoryview / numpy array /
// torch tensor derived from it is alive; the pin is dropped in the destructor,
// which is what lets the store defer freeing deleted-but-still-viewed objects.
struct PinnedBuffer {
  std::shared_ptr<ObjectStore> store;
  std::string id;
  uint64_t off, size, meta;
  ~PinnedBuffer() {
    if (store) store->unpin(id);
  }
};

PYBIND11_MODULE(_native, m) {
  m.doc() = "cluster_anywhere_amd native runtime (object store, scheduler)";

  py::class_<PinnedBuffer>(m, "PinnedBuffer", py::buffer_protocol())
      .def_buffer([](PinnedBuffer& b) -> py::buffer_info {
        return py::buffer_info(b.store->base() + b.off, 1, py::format_descriptor<uint8_t>::format(),
                               1, {(ssize_t)b.size}, {1}, /*readonly=*/true);
      })
      .def_readonly("size", &PinnedBuffer::size)
      .def_readonly("meta", &PinnedBuffer::meta);

  py::class_<ObjectStore, std::shared_ptr<ObjectStore>>(m, "ObjectStore")
      .def(py::init<const std::string&, uint64_t, uint64_t, bool>(), py::arg("name"),
           py::arg("capacity") = 0, py::arg("table_capacity") = 1 << 16, py::arg("create") = false)
      .def("create",
           [](ObjectStore& s, py::bytes id, uint64_t size, uint64_t meta) {
             py::gil_scoped_release g;
             return s.create(std::string(id), size, meta);
           },
           py::arg("id"), py::arg("size"), py::arg("meta") = 0)
      .def("seal", [](ObjectStore& s, py::bytes id) { return s.seal(std::string(id)); })
      .def("lookup",
           [](ObjectStore& s, py::bytes id, bool pin) -> py::object {
             uint64_t off, size, meta;
             if (!s.lookup(std::string(id), &off, &size, &meta, pin)) return py::none();
             return py::make_tuple(off, size, meta);
           },
           py::arg("id"), py::arg("pin") = false)
      .def("unpin", [](ObjectStore& s, py::bytes id) { s.unpin(std::string(id)); })
      .def("get_pinned",
           [](std::shared_ptr<ObjectStore> s, py::bytes id) -> py::object {
             uint64_t off, size, meta;
             std::string sid(id);
             if (!s->lookup(sid, &off, &size, &meta, true)) return py::none();
             auto pb = new PinnedBuffer{s, sid, off, size, meta};
             return py::cast(pb, py::return_value_policy::take_ownership);
           })
      .def("contains", [](ObjectStore& s, py::bytes id) { return s.contains(std::string(id)); })
      .def("remove", [](ObjectStore& s, py::bytes id) { return s.remove(std::string(id)); })
      .def("abort", [](ObjectStore& s, py::bytes id) { return s.abort(std::string(id)); })
      .def("buffer",
           [](ObjectStore& s, uint64_t off, uint64_t size, bool readonly) {
             return py::memoryview::from_memory(s.base() + off, (ssize_t)size, readonly);
           },
           py::arg("offset"), py::arg("size"), py::arg("readonly") = true)
      .def("address", [](ObjectStore& s, uint64_t off) { return (uintptr_t)(s.base() + off); })
      .def("lru_candidates",
           [](ObjectStore& s, uint64_t n) {
             std::vector<py::bytes> out;
             for (auto& x : s.lru_candidates(n)) out.emplace_back(x);
             return out;
           })
      .def("list_ids",
           [](ObjectStore& s) {
             std::vector<py::bytes> out;
             for (auto& x : s.list_ids()) out.emplace_back(x);
             return out;
           })
      .def("copy_in",
           [](ObjectStore& s, uint64_t off, py::buffer b, int threads) {
             py::buffer_info info = b.request();
             const uint64_t n = (uint64_t)(info.size * info.itemsize);
             if (off + n > s.map_size()) throw py::index_error("copy_in past the end of the arena");
             py::gil_scoped_release g;
             s.copy_in(off, info.ptr, n, threads);
           },
           py::arg("offset"), py::arg("data"), py::arg("threads") = 8)
      .def("copy_threads_claimed", &ObjectStore::copy_threads_claimed)
      .def("_debug_plant_claim", &ObjectStore::debug_plant_claim)
      .def("prefault_async", &ObjectStore::prefault_async)
      .def("largest_free", &ObjectStore::largest_free)
      .def("unlink", &ObjectStore::unlink)
      .def_property_readonly("capacity", &ObjectStore::capacity)
      .def_property_readonly("map_size", &ObjectStore::map_size)
      .def_property_readonly("used", &ObjectStore::used)
      .def_property_readonly("num_objects", &ObjectStore::num_objects)
      .def_property_readonly("name", &ObjectStore::name);

  py::class_<ClusterScheduler>(m, "ClusterScheduler")
      .def(py::init<double>(), py::arg("spread_threshold") = 0.5)
      .def("add_node", &ClusterScheduler::add_node)
      .def("remove_node", &ClusterScheduler::remove_node)
      .def("set_alive", &ClusterScheduler::set_alive)
      .def("total", &ClusterScheduler::total)
      .def("available", &ClusterScheduler::available)
      .def("cluster_total", &ClusterScheduler::cluster_total)
      .def("cluster_available", &ClusterScheduler::cluster_available)
      .def("nodes", &ClusterScheduler::nodes)
      .def("pick_node",
           [](ClusterScheduler& s, const ResMap& demand, int strategy, const std::string& aff, bool soft,
              const std::string& pref, const std::vector<std::tuple<std::string, int, std::vector<std::string>>>& hard,
              const std::vector<std::tuple<std::string, int, std::vector<std::string>>>& softl) {
             auto conv = [](const std::vector<std::tuple<std::string, int, std::vector<std::string>>>& v) {
               std::vector<LabelCond> out;
               for (auto& t : v) out.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t)});
               return out;
             };
             return s.pick_node(demand, strategy, aff, soft, pref, conv(hard), conv(softl));
           },
           py::arg("demand"), py::arg("strategy") = 0, py::arg("affinity_node") = "",
           py::arg("soft") = false, py::arg("preferred_node") = "",
           py::arg("hard") = std::vector<std::tuple<std::string, int, std::vector<std::string>>>{},
           py::arg("soft_labels") = std::vector<std::tuple<std::string, int, std::vector<std::string>>>{})
      .def("set_labels", &ClusterScheduler::set_labels)
      .def("labels", &ClusterScheduler::labels)
      .def("acquire", &ClusterScheduler::acquire)
      .def("release", &ClusterScheduler::release)
      .def("reserve_pg", &ClusterScheduler::reserve_pg)
      .def("remove_pg", &ClusterScheduler::remove_pg)
      .def("pg_feasible", &ClusterScheduler::pg_feasible);

  // Channel: timeouts in seconds (< 0 = wait forever); waits release the GIL.
  py::class_<Channel, std::shared_ptr<Channel>>(m, "Channel")
      .def(py::init<const std::string&, bool, uint32_t, uint32_t, uint64_t>(), py::arg("name"),
           py::arg("create") = false, py::arg("num_readers") = 1, py::arg("num_slots") = 2,
           py::arg("slot_bytes") = 1 << 20)
      .def("write",
           [](Channel& c, py::buffer b, uint64_t flags, double timeout) {
             py::buffer_info info = b.request();
             int rc;
             {
               py::gil_scoped_release g;
               rc = c.write(info.ptr, (uint64_t)(info.size * info.itemsize), flags, timeout);
             }
             if (rc == -1) throw py::value_error("timeout");  // mapped to TimeoutError in Python
             if (rc == -2) throw py::stop_iteration("channel closed");
             if (rc == -3) throw py::buffer_error("message larger than the channel slot");
           },
           py::arg("data"), py::arg("flags") = 0, py::arg("timeout") = -1.0)
      .def("read",
           [](Channel& c, uint32_t reader, double timeout) -> py::tuple {
             const uint8_t* data;
             uint64_t len, flags;
             int rc;
             {
               py::gil_scoped_release g;
               rc = c.begin_read(reader, &data, &len, &flags, timeout);
             }
             if (rc == -1) throw py::value_error("timeout");
             if (rc == -2) throw py::stop_iteration("channel closed");
             if (rc != 0) throw py::index_error("bad reader index");
             py::bytes out((const char*)data, (size_t)len);
             c.end_read(reader);
             return py::make_tuple(out, flags);
           },
           py::arg("reader") = 0, py::arg("timeout") = -1.0)
      .def("close", &Channel::close)
      .def("unlink", &Channel::unlink)
      .def_property_readonly("closed", &Channel::closed)
      .def_property_readonly("num_readers", &Channel::num_readers)
      .def_property_readonly("num_slots", &Channel::num_slots)
      .def_property_readonly("slot_bytes", &Channel::slot_bytes)
      .def_property_readonly("write_seq", &Channel::write_seq)
      .def("read_seq", &Channel::read_seq)
      .def_property_readonly("name", &Channel::name);

  py::class_<GcsStore>(m, "GcsStore")
      .def(py::init<const std::string&, bool>(), py::arg("path"), py::arg("fsync_each") = false)
      .def("put",
           [](GcsStore& s, const std::string& t, py::bytes k, py::bytes v) {
             std::string ks(k), vs(v);
             py::gil_scoped_release g;
             s.put(t, ks, vs);
           })
      .def("delete", [](GcsStore& s, const std::string& t, py::bytes k) { return s.del(t, std::string(k)); })
      .def("get",
           [](GcsStore& s, const std::string& t, py::bytes k) -> py::object {
             std::string v;
             if (!s.get(t, std::string(k), &v)) return py::none();
             return py::bytes(v);
           })
      .def("keys",
           [](GcsStore& s, const std::string& t) {
             py::list out;
             for (auto& k : s.keys(t)) out.append(py::bytes(k));
             return out;
           })
      .def("items",
           [](GcsStore& s, const std::string& t) {
             py::list out;
             for (auto& kv : s.items(t)) out.append(py::make_tuple(py::bytes(kv.first), py::bytes(kv.second)));
             return out;
           })
      .def("tables", &GcsStore::tables)
      .def("clear_table", &GcsStore::clear_table)
      .def("sync", &GcsStore::sync)
      .def("compact", &GcsStore::compact)
      .def("_inject_write_fault", &GcsStore::inject_write_fault)
      .def_property_readonly("log_bytes", &GcsStore::log_bytes)
      .def_property_readonly("live_bytes", &GcsStore::live_bytes)
      .def_property_readonly("records_replayed", &GcsStore::records_replayed)
      .def_property_readonly("torn_bytes_dropped", &GcsStore::torn_bytes_dropped)
      .def_property_readonly("path", &GcsStore::path);
}
